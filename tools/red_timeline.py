"""Diagnostic: timeline of ONE one-launch training tick (SWARM_F_TICK_REDUCE, csrc/swarm_red.h)
from the stamps build's s_memrealtime stamps (100 MHz, chip-wide): acting and TD block ends,
and the acting blocks' reduce roles (entry, act_pro gate, TD gate, sweep done, end).

    python tools/red_timeline.py [envs] [agents]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["SWARM_LIB_PATH"] = os.path.join(ROOT, "experiments-2025-acsos-marl-for-swarming-behaviors_amd",
                                            "libswarm_hip_stamps.so")
import numpy as np  # noqa: E402
import torch  # noqa: E402

import swarm_amd  # noqa: E402
from swarm_amd import _lib  # noqa: E402


def q(x):
    x = np.asarray(x, dtype=np.float64)
    return f"median {np.median(x):6.2f} max {x.max():6.2f}" if x.size else "-"


def main():
    _lib.load()
    raw = ctypes.CDLL(_lib.LIB_PATH)
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    w0 = torch.tensor(np.load(os.path.join(ROOT, "tests", "golden", "weights.npz"))["weights_go_to"][0])
    eng = swarm_amd.SwarmEngine("GoTo", N, B, seed=0, params=w0, batch=B, eps=0.05)
    print("tick_reduce", eng.tick_reduce)
    eng.reset()
    for _ in range(100):
        eng.act(push=True, full_out=False)
        eng.advance()
    eng.reset()
    for _ in range(5):
        eng.train_tick()
    n_act = (B + 3) // 4
    n_blocks = n_act + (B + 3) // 4
    buf = torch.zeros(n_blocks * 16 * 32, dtype=torch.int64, device="cuda")
    raw.swarm_dbg_stamps_tick(ctypes.c_void_p(buf.data_ptr()))
    for rep in range(3):
        buf.zero_()
        eng.train_tick()
        torch.cuda.synchronize()
        a = buf.cpu().numpy().reshape(n_blocks, 16, 32)
        act, td = a[:n_act, :4], a[n_act:, :4]
        t0 = min(act[..., 30][act[..., 30] > 0].min(), td[..., 8][td[..., 8] > 0].min())

        def us(x):
            return (x[x > 0] - t0) / 100.0
        print(f"tick {rep}: acting waves end {q(us(act[..., 31]))} us; TD waves start {q(us(td[..., 8]))}, "
              f"end {q(us(td[..., 9]))} us")
        roles = a[: min(n_act, 107), 0]   # wave 0 of each role block
        names = {15: "role entry", 16: "act_pro gate passed", 17: "TD gate passed", 18: "sweep done", 19: "role end"}
        for k, nm in names.items():
            col = roles[1:106, k]
            print(f"  column roles {nm:22s} {q(us(col))} us")
        for vb, nm in ((0, "copy role"), (106, "control role")):
            if vb < roles.shape[0]:
                r = roles[vb]
                print(f"  {nm:12s} " + ", ".join(f"{names[k]} {(r[k] - t0) / 100.0:.2f}" for k in (15, 16, 17, 19) if r[k] > 0))
    print("errors", eng.handoff_errors())


if __name__ == "__main__":
    main()
