"""Diagnostic (CPU only): how far a legitimate fp32 FORWARD moves the TD gradient, against the
per-tensor bound tests/test_gpu_parity_large.py had until round 6's last change.

That bound was 4x "the fp32 oracle's own error": the largest distance to the float64 evaluation of
four fp32 evaluations (the batch in three orders, and the other formulation); the evaluation below
is now the fifth member of that spread.  Three of the four
share torch's rounding of every per-node dot product, so Q's last bits, which the TD error
delta = Q - y amplifies (|Q| ~ 10^2, |delta| ~ 1), are nearly the same in all of them.  This tool
adds a fifth evaluation that differs only there: every linear layer correctly rounded
(oracle.swarm_oracle.correctly_rounded_linears) -- per dot product MORE accurate than torch's -- and
prints its distance to float64 as a multiple of the four-evaluation spread, per parameter tensor.

Data: C5's shard shapes (ObstacleAvoidance, N agents x 512 envs, S = 512 drawn from a 4-slot ring
of the oracle's own eps-greedy ticks from a reset formation; online weights = the reference's OA
seed 5 checkpoint, target = seed 6), as in test_td_api_update_at_benchmark_size.

usage: python tools/fwd_rounding.py [--out profiles/r06_fwd_rounding.json] [N ...]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import swarm_oracle as O  # noqa: E402


def ring(N, conv, B=512, slots=4):
    w = np.load(os.path.join(ROOT, "tests/golden/weights.npz"))["weights_obstacle_avoidance"]
    p, t = torch.tensor(w[5]), torch.tensor(w[6])
    P = O.unflatten_params(p)
    c = O.reset_centres(O.SCENARIO_OA, B, 12, 0, False)
    pos, vel = O.grid_positions(torch.as_tensor(c, dtype=torch.float32), N), torch.zeros(B, N, 2)
    s, a, r, s1 = [], [], [], []
    for k in range(slots):
        o = O.act_tick(P, pos, vel, O.SCENARIO_OA, O.GRAPH_COMPLETE, 0, 0.3, 12, k, conv=conv)
        s.append(torch.cat([pos, vel], -1))
        a.append(o.actions)
        r.append(o.step["rew"].to(torch.float32))
        pos, vel = o.step["pos"], o.step["vel"]
        s1.append(torch.cat([pos, vel], -1))
    return p, t, torch.cat(s), torch.cat(a), torch.cat(r), torch.cat(s1)


def case(N, conv, S=512):
    p, t, s, a, r, s1 = ring(N, conv)
    idx = torch.randperm(s.shape[0], generator=torch.Generator().manual_seed(S + N))[:S]
    s, a, r, s1 = s[idx], a[idx], r[idx], s1[idx]
    g64 = O.td_loss_grad(p, t, s, a, r, s1, conv=conv, dtype=torch.float64)[1]
    evals = []
    for q in (torch.arange(S), torch.arange(S - 1, -1, -1), torch.randperm(S, generator=torch.Generator().manual_seed(S + N))):
        evals.append(O.td_loss_grad(p, t, s[q], a[q], r[q], s1[q], conv=conv)[1])
    evals.append(O.td_loss_grad(p, t, s, a, r, s1, conv="gcn_edges" if conv == "gcn" else "gat_dense")[1])
    with O.correctly_rounded_linears():
        gcr = O.td_loss_grad(p, t, s, a, r, s1, conv=conv)[1]
    out, o = {}, 0
    for k, shape in O.PARAM_ORDER:
        n = int(np.prod(shape))
        b = g64[o:o + n]
        o += n
        if float(b.abs().max()) == 0.0:   # GCN: the attention vectors get no gradient
            continue
        spread = max(float((g[o - n:o].double() - b).abs().max()) for g in evals)
        e_cr = float((gcr[o - n:o].double() - b).abs().max())
        gmax = float(b.abs().max())
        bound = 4.0 * spread + 4.0 * float(torch.finfo(torch.float32).eps) * 2.0 ** np.floor(np.log2(gmax))
        out[k] = {"spread4": spread, "cr_error": e_cr, "cr_over_spread4": e_cr / spread,
                  "test_bound": bound, "cr_over_test_bound": e_cr / bound}
    worst = max(out.items(), key=lambda kv: kv[1]["cr_over_spread4"])
    return {"N": N, "conv": conv, "tensors": out, "worst_tensor": worst[0], "worst_ratio": worst[1]["cr_over_spread4"],
            "worst_over_test_bound": max(v["cr_over_test_bound"] for v in out.values())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("N", nargs="*", type=int, default=list(range(5, 13)))
    args = ap.parse_args()
    res = []
    for N in args.N:
        for conv in ("gat", "gcn"):
            d = case(N, conv)
            res.append(d)
            print(f"N={N:2d} {conv}: correctly-rounded-linear evaluation at {d['worst_ratio']:.2f}x the "
                  f"four-evaluation spread ({d['worst_tensor']}); {d['worst_over_test_bound']:.2f} of the tests' "
                  f"per-tensor bound", flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump({"tool": "tools/fwd_rounding.py", "bound_in_tests": "4x spread4 + 4 ulps", "cases": res}, f, indent=1)


if __name__ == "__main__":
    main()
