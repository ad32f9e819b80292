import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")
# agent counts of the recorded evaluation runs committed as fixtures (tests/golden/make_golden.py):
# every N the reference recorded, i.e. C5's whole 5-12 sweep (VERDICT r5 "next" #1)
RECORDED_AGENTS = tuple(range(5, 13))
# achieved errors of every numeric comparison, written at session end (record the
# observed margins, not just pass/fail) to gpurun_out/parity_errors.<kind>.json, kind = "gpu" when
# the session ran a test marked gpu, else "cpu": a CPU run never overwrites a GPU run's margins.
# The GPU runs copy the gpu file to profiles/.
ERRORS_DIR = os.path.join(ROOT, "gpurun_out")
_RECORDS = []
_RAN_GPU = []


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the built libswarm_hip.so")


def pytest_runtest_setup(item):
    if item.get_closest_marker("gpu") is not None:
        _RAN_GPU.append(item.nodeid)


def errors_path(ran_gpu: bool) -> str:
    return os.environ.get("SWARM_PARITY_ERRORS") or os.path.join(
        ERRORS_DIR, "parity_errors.%s.json" % ("gpu" if ran_gpu else "cpu"))


def pytest_sessionfinish(session, exitstatus):
    if not _RECORDS:
        return
    out = errors_path(bool(_RAN_GPU))
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as f:
        json.dump({"exitstatus": int(exitstatus), "kind": "gpu" if _RAN_GPU else "cpu", "records": _RECORDS}, f,
                  indent=0)


@pytest.fixture(scope="session")
def golden_weights():
    import numpy as np
    z = np.load(os.path.join(GOLDEN, "weights.npz"))
    f = np.load(os.path.join(GOLDEN, "flocking_weights.npz"))
    return {"go_to": z["weights_go_to"], "obstacle_avoidance": z["weights_obstacle_avoidance"],
            "flocking_gat3": f["weights_flocking"]}


@pytest.fixture(scope="session")
def trajectories():
    import numpy as np
    return np.load(os.path.join(GOLDEN, "trajectories.npz"))


def fp32_ulp(b):
    """spacing of fp32 at |b| (elementwise, float64 tensor); subnormal floor at 2^-126."""
    import numpy as np
    import torch
    x = np.abs(torch.as_tensor(b, dtype=torch.float64).cpu().numpy()).astype(np.float32)
    x = np.maximum(x, np.float32(2.0 ** -126))
    return torch.from_numpy(np.spacing(x).astype(np.float64))


def error_stats(a, b, scale=None):
    """max |a-b|, max |a-b|/max(1,|b|), max |a-b| in fp32 ulps of max(|b|, scale) (scale: an
    optional floor, e.g. the magnitude of the terms the value sums, for elements near 0)."""
    import torch
    a = torch.as_tensor(a, dtype=torch.float64).cpu().reshape(-1)
    b = torch.as_tensor(b, dtype=torch.float64).cpu().reshape(-1)
    if a.numel() == 0:
        return dict(n=0, max_abs=0.0, max_rel=0.0, max_ulp=0.0)
    err = (a - b).abs()
    ref = b.abs() if scale is None else torch.maximum(b.abs(), torch.as_tensor(scale, dtype=torch.float64).reshape(-1)
                                                     .expand_as(b))
    ulp = err / fp32_ulp(ref)
    return dict(n=int(a.numel()), max_abs=float(err.max()), max_rel=float((err / b.abs().clamp_min(1.0)).max()),
                max_ulp=float(ulp.max()), mean_ulp=float(ulp.mean()))


def record(what, stats, **extra):
    """Keep one comparison's achieved error for the session's parity_errors.json."""
    rec = {"test": os.environ.get("PYTEST_CURRENT_TEST", "").split(" ")[0], "what": what}
    rec.update(stats)
    rec.update(extra)
    _RECORDS.append(rec)
    return rec


def assert_close_rel(a, b, tol=1e-5, what=""):
    """north_star tolerance 'Q-values and TD-loss within 1e-5 fp32', applied relative to
    magnitude: |a - b| <= tol * max(1, |b|) elementwise (an fp32 ulp at |Q|~234 is 1.5e-5).
    The achieved error (absolute, relative, fp32 ulps) is recorded."""
    st = error_stats(a, b)
    record(what, st, tol_rel=tol)
    assert st["max_rel"] <= tol, f"{what}: max relative error {st['max_rel']:.3e} > {tol:.1e}"


def assert_close_ulp(a, b, max_ulp, what="", scale=None, rel_floor=None):
    """|a - b| <= max_ulp fp32 ulps of max(|b|, scale) elementwise; recorded.  ``rel_floor`` also
    keeps the north_star's 1e-5 relative bound as an upper limit (both must hold)."""
    st = error_stats(a, b, scale)
    record(what, st, tol_ulp=max_ulp)
    assert st["max_ulp"] <= max_ulp, f"{what}: {st['max_ulp']:.1f} ulp > {max_ulp} (max abs {st['max_abs']:.3e})"
    if rel_floor is not None:
        assert st["max_rel"] <= rel_floor, f"{what}: max relative error {st['max_rel']:.3e} > {rel_floor:.1e}"
