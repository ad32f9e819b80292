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

ACT = {0: "entry", 1: "prologue(state+params->LDS)", 2: "lin0+scores+H->LDS", 3: "barrier+graph_mult",
       4: "softmax+aggregate", 5: "tanh", 6: "lin1(MFMA)+relu", 7: "lin2(VALU)", 8: "eps-greedy(philox)",
       9: "agent_step(physics)", 10: "reward/metrics(LDS)", 11: "stores+barrier", 12: "end"}
TD = {0: "entry", 1: "params loads+ctrl+skip", 2: "sample_index(feistel)", 3: "replay loads+LDS stage+barrier",
      16: "fwd lin0+scores", 17: "barrier+graph_mult", 18: "softmax+aggregate", 19: "tanh", 20: "lin1",
      21: "lin2", 4: "(y)", 5: "barrier (y ready)", 6: "MLP backward (W2,relu,W1^T MFMA,tanh')",
      7: "image writes+barrier", 8: "GAT attn bwd | dW1,dW2,sums  +barrier", 9: "dh messages+barrier",
      10: "dW + datt", 11: "partial slab write+barrier", 12: "block slab sum+store"}


def report(buf, names, nwaves):
    a = buf.reshape(-1, 32)[:nwaves].astype(np.int64)
    order = sorted(names, key=lambda k: (k if k < 16 else 3.5 + (k - 16) * 0.01))
    order = [k for k in order if (a[:, k] > 0).all()]
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
        eng.train_tick()
    torch.cuda.synchronize()
    assert raw.swarm_dbg_stamps_act(sa.data_ptr()) == 0 and raw.swarm_dbg_stamps_td(st.data_ptr()) == 0
    for _ in range(3):
        eng.train_tick()
    torch.cuda.synchronize()
    tiles = (B + (32 // N) - 1) // (32 // N)
    ab = (tiles + 3) // 4
    print(f"act_kernel ({ab} blocks x 4 waves):")
    report(sa.cpu().numpy()[: ab * 16 * 32].reshape(ab, 16, 32)[:, :4].reshape(-1), ACT, ab * 4)
    tpb = int(os.environ.get("SWARM_TD_TPB", 1))
    blocks = (tiles + tpb - 1) // tpb
    td = st.cpu().numpy()[: blocks * 16 * 32].reshape(blocks, 16, 32)
    print(f"td_kernel ({blocks} blocks x {tpb} tiles), online waves:")
    report(td[:, :tpb].reshape(-1), TD, blocks * tpb)
    print("td_kernel target waves:")
    report(td[:, tpb:2 * tpb].reshape(-1), TD, blocks * tpb)


if __name__ == "__main__":
    main()
