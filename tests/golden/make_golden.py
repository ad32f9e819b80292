"""Build the committed golden fixtures from the reference's own recorded outputs.

Run in the build container (``/root/reference`` is read-only and absent on the
GPU box):  ``python tests/golden/make_golden.py``.

Sources (all data files the reference ships; no reference code is executed):

* ``data/models/experiment_{GoTo,ObstacleAvoidance}-seed_{0..9}.pth`` — trained
  ``GCN`` state_dicts, loaded with ``torch.load(weights_only=True)`` and
  flattened in ``state_dict`` order (``oracle.swarm_oracle.PARAM_ORDER``).
* ``data/test_stats/{go_to,obstacle_avoidance}/seed_{s}/agents_{n}/`` — per-tick
  positions (``positions/positions_episode_{e}_{x,y}.csv``), per-tick average
  distance and hits (``data/distances_episode_{e}.csv``) and per-episode
  ``result.csv``, written by ``src/simulation/simulator.py:111-166`` with kNN k=5
  (SURVEY.md §4, §8(c)).

Derived per tick t (1 <= t <= T-2), using only recorded positions P:
  V_t = (P_t - P_{t-1}) / 0.1 ;  F_{t+1} = (V_{t+1} - 0.75 V_t) / 0.1 = u_t + f_coll(P_t)
``ref_action[t]`` = the discrete action whose decode u equals
round(F_{t+1} - f_coll(P_t)); it is the action the reference's policy took at t.

Also writes ``topk_ties.npz``: tie-heavy distance rows with the index sets that
this container's CPU ``torch.topk(largest=False)`` selects (the reference's call
at ``simulator.py:19``; torch 2.10 here vs 2.6 pinned — same nth_element path).
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import swarm_oracle as O  # noqa: E402

REF = "/root/reference/data"
SCEN = [("go_to", O.SCENARIO_GOTO, "GoTo"), ("obstacle_avoidance", O.SCENARIO_OA, "ObstacleAvoidance")]
SEEDS = (0, 4)
AGENTS = tuple(range(5, 13))   # every agent count the reference recorded (C5 sweeps 5-12)
EPISODES = 8
LEVEL_IDX = {0: 0, -1: 1, 1: 2}


def load_positions(scen, seed, n, ep):
    d = f"{REF}/test_stats/{scen}/seed_{seed}/agents_{n}/positions"
    X = np.loadtxt(f"{d}/positions_episode_{ep}_x.csv", delimiter=",", skiprows=1)[:, 1:]
    Y = np.loadtxt(f"{d}/positions_episode_{ep}_y.csv", delimiter=",", skiprows=1)[:, 1:]
    P = np.stack([X, Y], -1)
    P32 = P.astype(np.float32)
    assert np.array_equal(P32.astype(np.float64), P), "recorded positions are fp32 values"
    return P32


def ref_actions(P32, scenario):
    P = P32.astype(np.float64)
    T, N, _ = P.shape
    V = np.zeros_like(P)
    V[1:] = (P[1:] - P[:-1]) / 0.1
    acts = np.full((T, N), -1, dtype=np.int8)
    for t in range(1, T - 1):
        F = (V[t + 1] - 0.75 * V[t]) / 0.1
        pos = torch.tensor(P32[t])[None]
        zero = torch.zeros(1, N, dtype=torch.long)  # action 0 -> u=0, so force = f_coll
        fcoll = O.env_step(pos, torch.zeros(1, N, 2), zero, scenario)["force"][0].double().numpy()
        u = F - fcoll
        ur = np.rint(u)
        if np.abs(u - ur).max() > 1e-3 or np.abs(ur).max() > 1:
            raise RuntimeError("non-integral recorded action")
        for i in range(N):
            acts[t, i] = 3 * LEVEL_IDX[int(ur[i, 0])] + LEVEL_IDX[int(ur[i, 1])]
    return acts


def main():
    out = {}
    for scen, _, mname in SCEN:
        W = []
        for s in range(10):
            sd = torch.load(f"{REF}/models/experiment_{mname}-seed_{s}.pth", weights_only=True)
            W.append(O.flatten_params(sd).numpy())
        out[f"weights_{scen}"] = np.stack(W).astype(np.float32)
    np.savez_compressed(os.path.join(HERE, "weights.npz"), **out)

    traj = {}
    for scen, sid, _ in SCEN:
        for seed in SEEDS:
            for n in AGENTS:
                base = f"{REF}/test_stats/{scen}/seed_{seed}/agents_{n}"
                res = np.loadtxt(f"{base}/result.csv", delimiter=",", skiprows=1)
                traj[f"{scen}/s{seed}/n{n}/result"] = res.astype(np.float64)
                for ep in range(EPISODES):
                    P = load_positions(scen, seed, n, ep)
                    dist = np.loadtxt(f"{base}/data/distances_episode_{ep}.csv", delimiter=",", skiprows=1)
                    key = f"{scen}/s{seed}/n{n}/e{ep}"
                    traj[key + "/pos"] = P
                    traj[key + "/dist"] = dist[:, 1].astype(np.float64)
                    traj[key + "/hits"] = dist[:, 2].astype(np.float64)
                    traj[key + "/ref_action"] = ref_actions(P, sid)
    np.savez_compressed(os.path.join(HERE, "trajectories.npz"), **traj)

    # topk tie vectors: grid-like rows with exact ties
    rng = np.random.default_rng(1234)
    rows, ks, sets = [], [], []
    for _ in range(3000):
        n = int(rng.integers(5, 17))
        k = int(rng.integers(1, n + 1))
        kind = rng.integers(0, 3)
        if kind == 0:      # lattice distances -> many exact ties
            d = rng.integers(0, 4, size=n).astype(np.float32) * np.float32(0.15)
        elif kind == 1:    # few distinct values
            vals = rng.random(3).astype(np.float32)
            d = vals[rng.integers(0, 3, size=n)]
        else:              # from a real grid formation with one displaced agent
            offs = O.grid_offsets(n).astype(np.float32)
            c = rng.normal(size=2).astype(np.float32)
            p = torch.tensor(offs + c)
            if rng.random() < 0.5:
                p[rng.integers(0, n)] += torch.tensor(rng.normal(scale=0.05, size=2).astype(np.float32))
            i = int(rng.integers(0, n))
            d = torch.linalg.norm(p - p[i], dim=1).numpy()
        _, idx = torch.topk(torch.tensor(d), k, largest=False)
        s = np.zeros(16, dtype=np.uint8)
        s[idx.numpy()] = 1
        row = np.full(16, np.inf, dtype=np.float32)
        row[:n] = d
        rows.append(row)
        ks.append((n, k))
        sets.append(s)
    np.savez_compressed(os.path.join(HERE, "topk_ties.npz"), dist=np.stack(rows),
                        nk=np.asarray(ks, dtype=np.int32), sets=np.stack(sets))
    print("wrote", sorted(os.listdir(HERE)))


if __name__ == "__main__":
    main()
