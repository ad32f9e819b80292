"""Diagnostic: per-segment cycle shares of act_kernel / td_kernel from in-kernel
s_memtime stamps (libswarm_hip_stamps.so, -DSWARM_STAMPS=1).  Read the SHARES;
the stamp build itself runs slower than the real one."""
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

FWD = {0: "fwd lin0 + scores + H image", 1: "fwd softmax coefficients", 2: "fwd aggregate MFMA + tanh",
       3: "fwd lin1 MFMA", 4: "fwd lin2 MFMA + Q exchange"}
ACT = {0: "entry", 20: "pro: loads issued + ctrl", 21: "pro: norm partials (data arrival)",
       22: "pro: norm reduction (barrier)", 23: "pro: Adam elements", 24: "pro: w -> LDS",
       1: "pro: barrier", **{8 + k: v for k, v in FWD.items()},
       2: "(end of forward)",
       5: "argmax + eps-greedy", 6: "pair forces -> LDS", 7: "wave LDS sync", 3: "force sum + integrate + aux",
       13: "sync + goal distances -> reward", 14: "stores", 4: "state store + TD batch draw"}
TD = {0: "entry", 1: "params loads + ctrl + skip + sample index", 2: "replay loads + LDS stage + barrier",
      **{16 + k: v for k, v in FWD.items()}, 3: "(y)", 4: "barrier (y ready)", 5: "dQ/dZ images + barrier",
      24: "bwd: dT MFMA + dO images", 25: "bwd: GAT g MFMA / dp + sync",
      27: "bwd: da_src + dh messages MFMA + dH images",
      6: "(online: B3 barrier) | target: dW1,dW2,b1 products + B3", 7: "dW / att / bias products"}


ACT_ORDER = [0, 20, 21, 22, 23, 24, 1, 8, 9, 10, 11, 12, 2, 5, 6, 7, 3, 13, 14, 4]
TD_ORDER = [0, 1, 2, 16, 17, 18, 19, 20, 3, 4, 5, 24, 25, 27, 6, 7]


def rt_window(buf, nwaves, first, last):
    """(start, end) of a launch in s_memrealtime ticks (100 MHz, chip-wide): earliest entry
    stamp, latest exit stamp over the waves that wrote both."""
    a = buf.reshape(-1, 32)[:nwaves].astype(np.int64)
    a = a[(a[:, first] > 0) & (a[:, last] > 0)]
    st = a[:, first]
    print(f"  launch span {(a[:, last].max() - st.min()) / 100:.2f} us; wave entries spread "
          f"{np.percentile(st - st.min(), 50) / 100:.2f} (median) / {(st.max() - st.min()) / 100:.2f} (max) us; "
          f"wave exits spread {(a[:, last].max() - np.percentile(a[:, last], 50)) / 100:.2f} us after the median")
    return st.min(), a[:, last].max()


def report(buf, names, nwaves, order):
    a = buf.reshape(-1, 32)[:nwaves].astype(np.int64)
    order = [k for k in order if k in names and (a[:, k] > 0).all()]
    tot = np.median(a[:, order[-1]] - a[:, order[0]])
    print(f"  total median {tot:.0f} cycles")
    for p, k in zip(order, order[1:]):
        d = np.median(a[:, k] - a[:, p])
        print(f"  {names[k]:42s} {d:8.0f} cyc  {100 * d / tot:5.1f}%")


def main():
    lib = _lib.load()
    raw = ctypes.CDLL(_lib.LIB_PATH)
    B, N = int(os.environ.get("ENVS", 1024)), int(os.environ.get("AGENTS", 8))
    w = torch.tensor(np.load(os.path.join(ROOT, "tests/golden/weights.npz"))["weights_go_to"][0])
    eng = swarm_amd.SwarmEngine("GoTo", N, B, seed=0, params=w, batch=B, eps=0.05)
    sa = torch.zeros(4096 * 16 * 32, dtype=torch.int64, device="cuda")
    st = torch.zeros_like(sa)
    raw.swarm_dbg_stamps_act.argtypes = [ctypes.c_void_p]
    raw.swarm_dbg_stamps_td.argtypes = [ctypes.c_void_p]
    eng.reset(0)
    for _ in range(30):
        eng.train_tick3()
    torch.cuda.synchronize()
    assert raw.swarm_dbg_stamps_act(sa.data_ptr()) == 0 and raw.swarm_dbg_stamps_td(st.data_ptr()) == 0
    graph = eng.capture(3, lambda: eng.train_tick3(full_out=False))   # the 3-launch tick (same act / TD bodies)
    graph.replay()
    torch.cuda.synchronize()
    ab = (B + 3) // 4
    print(f"act_kernel ({ab} blocks x 4 waves, one env per wave):")
    report(sa.cpu().numpy()[: ab * 16 * 32].reshape(ab, 16, 32)[:, :4].reshape(-1), ACT, ab * 4, ACT_ORDER)
    wa = rt_window(sa.cpu().numpy()[: ab * 16 * 32].reshape(ab, 16, 32)[:, :4].reshape(-1), ab * 4, 30, 31)
    ns = 16 if N <= 16 else 32          # node slots per TD wave (two 8-slot graphs when N <= 8)
    gs = 8 if N <= 8 else ns
    gpb = 32 // ns                      # online (= target) waves per block
    blocks = (B + 32 // gs - 1) // (32 // gs)
    td = st.cpu().numpy()[: blocks * 16 * 32].reshape(blocks, 16, 32)
    print(f"td_kernel ({blocks} blocks x {gpb} online + {gpb} target waves), online waves:")
    report(td[:, :gpb].reshape(-1), TD, blocks * gpb, TD_ORDER)
    wt = rt_window(td[:, :2 * gpb].reshape(-1), blocks * 2 * gpb, 8, 9)
    print("td_kernel target waves:")
    report(td[:, gpb:2 * gpb].reshape(-1), TD, blocks * gpb, TD_ORDER)
    nrb, own = (1674 + 15) // 16, 1673 // 16          # grad_reduce blocks (16 columns each), owner block
    red = st.cpu().numpy()[: nrb * 16 * 32].reshape(nrb, 16, 32)
    RED = {28: "entry", 29: "slab loads + partial sums", 30: "LDS combine + barrier", 31: "final sum, copy-back, ctrl/samples"}
    print("grad_reduce_kernel (advance), ordinary blocks:")
    report(red[:own].reshape(-1), RED, own * 16, [28, 29, 30, 31])
    wr = rt_window(red.reshape(-1), nrb * 16, 22, 23)
    print("grad_reduce_kernel owner block (ctrl + next-tick samples):")
    report(red[own:own + 1].reshape(-1), RED, 16, [28, 29, 30, 31])
    print(f"gaps (last exit -> first entry): act->td {(wt[0] - wa[1]) / 100:.2f} us, "
          f"td->reduce {(wr[0] - wt[1]) / 100:.2f} us; tick act entry -> reduce exit {(wr[1] - wa[0]) / 100:.2f} us")


if __name__ == "__main__":
    main()
