"""Diagnostic: accuracy of the GPU's Q-values against the oracle evaluated in float64, beside the
fp32 oracle's own, on replay-like states (OA, a reset formation plus a few eps-greedy ticks).

The TD error delta = Q - y cancels most of Q's magnitude (|Q| ~ 10^2, |delta| ~ 1), so the
gradient's accuracy is set by Q's ABSOLUTE error, and a bias (a mean signed error) adds up over
the batch instead of averaging out.  Prints mean |error| and mean signed error in fp32 ulps of Q.

usage: python tools/q_accuracy.py [N conv ...]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import swarm_amd  # noqa: E402
from swarm_amd import _lib  # noqa: E402
from swarm_amd.engine import ctypes_ref  # noqa: E402
from oracle import swarm_oracle as O  # noqa: E402


def states(N, conv, B=512):
    w = O.unflatten_params(torch.tensor(np.load(os.path.join(ROOT, "tests/golden/weights.npz"))
                                        ["weights_obstacle_avoidance"][5]))
    c = O.reset_centres(O.SCENARIO_OA, B, 12, 0, False)
    pos, vel = O.grid_positions(c, N), torch.zeros(B, N, 2)
    out = []
    for k in range(4):
        o = O.act_tick(w, pos, vel, O.SCENARIO_OA, O.GRAPH_COMPLETE, 0, 0.3, 12, k, conv=conv)
        pos, vel = o.step["pos"], o.step["vel"]
        out.append((pos, vel))
    return out


def main():
    args = sys.argv[1:] or ["12", "gcn", "12", "gat", "8", "gat", "5", "gcn"]
    p = torch.tensor(np.load(os.path.join(ROOT, "tests/golden/weights.npz"))["weights_obstacle_avoidance"][5])
    for N, conv in zip(args[0::2], args[1::2]):
        N = int(N)
        eng = swarm_amd.SwarmEngine("ObstacleAvoidance", N, 512, seed=1, params=p, conv=conv, learn=False)
        rows = []
        for pos, vel in states(N, conv):
            x = O.node_features(pos, vel)
            mult = O.multiplicity_complete(512, N)
            params = O.unflatten_params(p)
            if conv == "gat":
                q32 = O.q_forward_dense(params, x, mult)
                q64 = O.q_forward_dense({k: v.double() for k, v in params.items()}, x.double(), mult.double())
            else:
                q32 = O.gcn_conv_dense(params, x, mult)
                q64 = O.gcn_conv_dense({k: v.double() for k, v in params.items()}, x.double(), mult.double())
            qg = torch.zeros(512 * N, 9, device="cuda")
            xg = x.reshape(-1, 7).contiguous().cuda()
            _lib.check(eng.lib.swarm_q_forward(ctypes_ref(eng.cfg), eng.params.data_ptr(), xg.data_ptr(), None,
                                               qg.data_ptr(), _lib.stream_ptr()), "swarm_q_forward")
            torch.cuda.synchronize()
            qg = qg.cpu().reshape(512, N, 9).double()
            ulp = torch.from_numpy(np.spacing(np.abs(q64.numpy()).astype(np.float32)).astype(np.float64))
            rows.append(((qg - q64) / ulp, (q32.double() - q64) / ulp))
        eg = torch.cat([r[0].reshape(-1) for r in rows])
        eo = torch.cat([r[1].reshape(-1) for r in rows])
        print(f"OA N={N} {conv}: GPU mean|err| {eg.abs().mean():.3f} ulp, mean err {eg.mean():+.3f}, max {eg.abs().max():.1f}; "
              f"oracle32 mean|err| {eo.abs().mean():.3f}, mean err {eo.mean():+.3f}, max {eo.abs().max():.1f}")


if __name__ == "__main__":
    main()
