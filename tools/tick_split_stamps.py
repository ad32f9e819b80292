"""Where the un-profiled training tick goes: kernel spans and launch boundaries from in-kernel
s_memrealtime stamps (100 MHz, one clock for every XCD) of the realtime-stamps build
(libswarm_hip_rtstamps.so: a handful of stamps per wave, no segment stamps), with no profiler
attached.

The fused tick is two launches, tick_kernel then grad_reduce_kernel (swarm_reduce_advance).  A
launch's span runs from its first wave's entry stamp to its last wave's exit stamp; the gap from
one launch's last exit to the next launch's first entry is the launch boundary (end-of-kernel
cache release, the CP's next dispatch, wave launch).  Each (block, wave) stamp slot keeps the last
launch that wrote it, so two captured sequences are replayed (after warm ticks, in steady state):

  [tick, reduce]          -> tick span, tick -> reduce boundary, reduce span
  [tick, reduce, tick]    -> the reduce -> next tick boundary (reduce slots hold launch 2, tick
                             slots launch 3)

and the four parts are compared with the tick period of a captured 100-tick chain of the same
library (HIP events).  `--lib=stamps` uses the segment-stamps build instead (much slower).

usage: python tools/tick_split_stamps.py [B N [GoTo|ObstacleAvoidance [gat|gcn]]] > out.txt
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# SWARM_SPLIT_LIB: a prebuilt realtime-stamps library to run instead (e.g. a diagnostic worktree's)
os.environ["SWARM_LIB_PATH"] = os.environ.get("SWARM_SPLIT_LIB") or os.path.join(
    ROOT, "experiments-2025-acsos-marl-for-swarming-behaviors_amd",
    "libswarm_hip_stamps.so" if "--lib=stamps" in sys.argv else "libswarm_hip_rtstamps.so")
sys.argv = [a for a in sys.argv if not a.startswith("--lib=")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import swarm_amd  # noqa: E402
from swarm_amd import _lib  # noqa: E402

RED_BLOCKS = (1674 + 15) // 16 + 1 + 3   # column blocks, control block, copy-back blocks


def span(a, first, last):
    """(first entry, last exit) in 100 MHz ticks over the waves that wrote both stamps."""
    a = a.reshape(-1, 32).astype(np.int64)
    a = a[(a[:, first] > 0) & (a[:, last] > 0)]
    return int(a[:, first].min()), int(a[:, last].max())


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    scen = sys.argv[3] if len(sys.argv) > 3 else "GoTo"
    conv = sys.argv[4] if len(sys.argv) > 4 else "gat"
    _lib.load()
    raw = ctypes.CDLL(_lib.LIB_PATH)
    raw.swarm_dbg_stamps_tick.argtypes = [ctypes.c_void_p]
    raw.swarm_dbg_stamps_td.argtypes = [ctypes.c_void_p]
    key = "weights_go_to" if scen == "GoTo" else "weights_obstacle_avoidance"
    w0 = torch.tensor(np.load(os.path.join(ROOT, "tests", "golden", "weights.npz"))[key][0])
    eng = swarm_amd.SwarmEngine(scen, N, B, seed=0, params=w0, batch=B, eps=0.05, conv=conv)
    assert eng.fused
    eng.reset()
    for _ in range(100):
        eng.act(push=True, full_out=False)
        eng.advance()
    eng.reset()
    n_act = (B + 3) // 4
    n_td = (B + 3) // 4 if N <= 8 else (B + 1) // 2
    tbuf = torch.zeros((n_act + n_td) * 16 * 32, dtype=torch.int64, device="cuda")
    rbuf = torch.zeros(max(RED_BLOCKS, n_td) * 16 * 32, dtype=torch.int64, device="cuda")
    assert raw.swarm_dbg_stamps_tick(tbuf.data_ptr()) == 0 and raw.swarm_dbg_stamps_td(rbuf.data_ptr()) == 0

    def tick():
        eng.launch_tick()
        eng.launch_reduce_advance()

    g_pair = eng.capture(1, tick)
    g_rt = eng.capture(1, lambda: (eng.launch_tick(), eng.launch_reduce_advance(), eng.launch_tick()))
    g_chain = eng.capture(100, tick)
    stream = torch.cuda.current_stream()
    res = {"B": B, "N": N, "scenario": scen, "conv": conv, "library": _lib.load().swarm_build_info().decode()}
    rows, gap_rt = [], []
    for rep in range(5):
        for _ in range(3):
            tick()
        tbuf.zero_()
        rbuf.zero_()
        g_pair.replay()
        torch.cuda.synchronize()
        t = tbuf.cpu().numpy().reshape(n_act + n_td, 16, 32)
        r = rbuf.cpu().numpy().reshape(-1, 16, 32)[:RED_BLOCKS]
        a0, a1 = span(t[:n_act, :4], 30, 31)
        d0, d1 = span(t[n_act:, :4], 8, 9)
        r0, r1 = span(r, 22, 23)
        k0, k1 = min(a0, d0), max(a1, d1)
        rows.append({"tick_span_us": (k1 - k0) / 100, "tick_to_reduce_gap_us": (r0 - k1) / 100,
                     "reduce_span_us": (r1 - r0) / 100, "act_waves_us": (a1 - a0) / 100,
                     "td_waves_us": (d1 - d0) / 100})
        # per block kind, when the library stamps the control and copy-back blocks' exits too: the
        # last exit of the column blocks, the control block and the copy-back blocks after r0
        ncol = RED_BLOCKS - 4
        kinds = {"columns": r[:ncol], "control": r[ncol:ncol + 1], "copy_back": r[ncol + 1:RED_BLOCKS]}
        for name, rr in kinds.items():
            a = rr.reshape(-1, 32).astype(np.int64)
            a = a[(a[:, 22] > 0) & (a[:, 23] > 0)]
            if len(a):
                rows[-1][f"reduce_{name}_end_us"] = (int(a[:, 23].max()) - r0) / 100
        # [tick, reduce, tick]: the reduce slots hold the middle launch, the tick slots the last
        tbuf.zero_()
        rbuf.zero_()
        g_rt.replay()
        torch.cuda.synchronize()
        t = tbuf.cpu().numpy().reshape(n_act + n_td, 16, 32)
        r = rbuf.cpu().numpy().reshape(-1, 16, 32)[:RED_BLOCKS]
        _, r1 = span(r, 22, 23)
        a0, _ = span(t[:n_act, :4], 30, 31)
        d0, _ = span(t[n_act:, :4], 8, 9)
        gap_rt.append((min(a0, d0) - r1) / 100)
        eng.launch_reduce_advance()   # completes the last tick (after the stamps were read)
        torch.cuda.synchronize()
    per = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        g_chain.replay()
        e1.record(stream)
        torch.cuda.synchronize()
        per.append(e0.elapsed_time(e1) * 1e3 / 100)
    med = {k: float(np.median([r[k] for r in rows if k in r])) for k in rows[0]}
    med["reduce_to_tick_gap_us"] = float(np.median(gap_rt))
    med["sum_us"] = med["tick_span_us"] + med["tick_to_reduce_gap_us"] + med["reduce_span_us"] + med["reduce_to_tick_gap_us"]
    med["tick_period_chain_us (HIP events, this library)"] = float(np.median(per))
    res["median_of_5"] = {k: round(v, 3) for k, v in med.items()}
    res["runs"] = rows
    res["reduce_to_tick_gaps_us"] = gap_rt
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
