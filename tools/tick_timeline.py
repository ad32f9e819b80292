"""Diagnostic: timeline of ONE fused training tick (swarm_train_tick) from in-kernel
s_memrealtime stamps (100 MHz, chip-wide) of the stamps build (libswarm_hip_stamps.so):
when the acting waves end, when the TD waves whose graphs come from the tick's own replay
slot get their hand-off, when the TD waves end.  Times in us from the first wave's entry.

usage: python tools/tick_timeline.py [B N [GoTo|ObstacleAvoidance [gat|gcn]]]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# SWARM_TL_LIB: a prebuilt stamps library to run instead (e.g. a diagnostic variant from
# tools/ab_build.py with -DSWARM_STAMPS=1); the in-tree stamps build otherwise
TL_LIB = os.environ.get("SWARM_TL_LIB")
os.environ["SWARM_LIB_PATH"] = TL_LIB or os.path.join(ROOT, "experiments-2025-acsos-marl-for-swarming-behaviors_amd",
                                                      "libswarm_hip_stamps.so")
import numpy as np  # noqa: E402
import torch  # noqa: E402

import swarm_amd  # noqa: E402
from swarm_amd import _lib  # noqa: E402
from tools.stamps import ACT, ACT_ORDER, TD, TD_ORDER, report  # noqa: E402

# stamp 10 (granules matched) is a 100 MHz realtime stamp, reported in us above.  The online
# waves of hand-off graphs take the pre path (swarm_tdk.h): their s wait follows B0 and leads the
# forward's first segment, their a wait and gq-free backward (dT, g, dp) come before y
TD_WAIT = {**TD, 2: "Adam + B0 barrier", 16: "s hand-off wait + " + TD[16],
           3: "a wait + pre path (dT, g MFMA, dp) + r wait + (y)", 5: "dQ/dZ + scaled dO/dp images + B2",
           25: "(pre path: nothing)", 26: "B2 jobs (pre online: vector sums)", 6: "B3 barrier wait"}
TD_WAIT_ORDER = [0, 1, 2, 16, 17, 18, 19, 20, 3, 4, 5, 25, 27, 26, 6, 7]


def main():
    from swarm_amd import build as swbuild
    if not TL_LIB:
        swbuild.build(stamps=True)
    lib = _lib.load()
    raw = ctypes.CDLL(_lib.LIB_PATH)
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    scen = sys.argv[3] if len(sys.argv) > 3 else "GoTo"
    conv = sys.argv[4] if len(sys.argv) > 4 else "gat"
    key = "weights_go_to" if scen == "GoTo" else "weights_obstacle_avoidance"
    w0 = torch.tensor(np.load(os.path.join(ROOT, "tests", "golden", "weights.npz"))[key][0])
    eng = swarm_amd.SwarmEngine(scen, N, B, seed=0, params=w0, batch=B, eps=0.05, conv=conv)
    eng.reset()
    for _ in range(100):
        eng.act(push=True, full_out=False)
        eng.advance()
    eng.reset()
    for _ in range(5):
        eng.train_tick()
    n_act = (B + 3) // 4
    n_blocks = n_act + (B + 3) // 4 if N <= 8 else n_act + (B + 1) // 2
    buf = torch.zeros(n_blocks * 16 * 32, dtype=torch.int64, device="cuda")
    raw.swarm_dbg_stamps_tick(ctypes.c_void_p(buf.data_ptr()))
    for rep in range(3):
        buf.zero_()
        eng.train_tick()
        torch.cuda.synchronize()
        a = buf.cpu().numpy().reshape(n_blocks, 16, 32)
        act = a[:n_act, :4]
        td = a[n_act:, :4]
        t0 = min(act[..., 30][act[..., 30] > 0].min(), td[..., 8][td[..., 8] > 0].min())
        us = lambda x: (x - t0) / 100.0  # noqa: E731
        ae = us(act[..., 31][act[..., 31] > 0])
        te = us(td[..., 9][td[..., 9] > 0])
        ts = us(td[..., 8][td[..., 8] > 0])
        pub = us(act[..., 29][act[..., 29] > 0])   # hand-off waves: s' published
        ho = td[..., 10]
        blocks_waiting = np.where((ho > 0).any(axis=1))[0]
        print(f"tick {rep}: act waves end median {np.median(ae):.2f} max {ae.max():.2f} us; "
              f"TD waves start median {np.median(ts):.2f}, end median {np.median(te):.2f} max {te.max():.2f} us")
        print(f"  {len(pub)} acting waves published s' (at {np.sort(pub).round(2).tolist()[:12]} us)")
        for b in blocks_waiting[:12]:
            on = us(ho[b, :2][ho[b, :2] > 0])
            tg = us(ho[b, 2:][ho[b, 2:] > 0])
            print(f"  TD block {b}: s matched {on.round(2).tolist()} us, s' matched {tg.round(2).tolist()} us, "
                  f"block end {us(td[b, :, 9].max()):.2f} us")
        other = np.setdiff1d(np.arange(td.shape[0]), blocks_waiting)
        oe = us(td[other][..., 9][td[other][..., 9] > 0])
        print(f"  TD blocks without hand-offs: waves end p50 {np.median(oe):.2f} p99 {np.percentile(oe, 99):.2f} "
              f"max {oe.max():.2f} us")
        nw = te[te > np.percentile(te, 99)]
        print(f"  slowest 1% TD waves end at {np.sort(nw).round(2).tolist()[-6:]} us")
        if rep == 2:   # per-segment medians (s_memtime cycles) of the critical waves
            print("  acting waves:")
            report(act.reshape(-1), ACT, act.shape[0] * 4, ACT_ORDER)
            wv = td[:, :2].reshape(-1, 32)   # online waves (2 per block at N <= 8)
            wv = wv[wv[:, 10] > 0]            # ... of waiting graphs
            if len(wv):
                print(f"  online TD waves of hand-off graphs ({len(wv)}):")
                report(wv.reshape(-1), TD_WAIT, len(wv), TD_WAIT_ORDER)
            tv = td[:, 2:].reshape(-1, 32)   # target waves of blocks with hand-off graphs
            tv = tv[tv[:, 10] > 0]
            if len(tv):
                print(f"  target TD waves of hand-off graphs ({len(tv)}):")
                report(tv.reshape(-1), {**TD, 2: "Adam + B0 barrier", 16: "s' hand-off wait + " + TD[16],
                                        3: "(y)", 26: "B2 jobs (dW1 / dW2 MFMA products)",
                                        6: "B3 barrier wait"},
                       len(tv), [0, 1, 2, 16, 17, 18, 19, 20, 3, 4, 5, 26, 6, 7])
            # the other online wave of a hand-off block (its graphs come from earlier slots): its
            # whole backward runs after B1, beside the pre wave's remainder and the target tiles
            npw = td[blocks_waiting, :2].reshape(-1, 32)
            npw = npw[npw[:, 10] == 0]
            if len(npw):
                print(f"  online TD waves without a hand-off graph, in hand-off blocks ({len(npw)}):")
                report(npw.reshape(-1), {**TD, 2: "Adam + B0 barrier", 26: "(no B2 jobs)", 6: "B3 barrier wait"},
                       len(npw), [0, 1, 2, 16, 17, 18, 19, 20, 3, 4, 5, 24, 25, 27, 26, 6, 7])
            print("  B2 -> arrival at B3 (stamps 5 -> 26), median cycles: " + ", ".join(
                f"{k} {np.median(x[:, 26] - x[:, 5]):.0f}" for k, x in
                (("pre online", wv), ("other online", npw), ("target", tv)) if len(x)))


if __name__ == "__main__":
    main()
