import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the built libswarm_hip.so")


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


def assert_close_rel(a, b, tol=1e-5, what=""):
    """north_star tolerance 'Q-values and TD-loss within 1e-5 fp32', applied relative to
    magnitude: |a - b| <= tol * max(1, |b|) elementwise (an fp32 ulp at |Q|~234 is 1.5e-5)."""
    import torch
    a = torch.as_tensor(a, dtype=torch.float64).cpu()
    b = torch.as_tensor(b, dtype=torch.float64).cpu()
    err = (a - b).abs() / b.abs().clamp_min(1.0)
    m = float(err.max()) if err.numel() else 0.0
    assert m <= tol, f"{what}: max relative error {m:.3e} > {tol:.1e}"
