"""CPU baseline loops for bench.py's ``cpu_baseline`` leg (TEST/BENCH INFRASTRUCTURE ONLY).

The reference itself cannot run here (vmas / torch_geometric absent),
so the CPU path is this oracle ("port"), timed on the host's cores:

* ``vectorized_train`` — the [B, N] oracle at the bench workload's shape: fused tick
  (dense GAT forward, ε-greedy, VMAS-order env step, replay push) + one TD update on
  S sampled graphs through torch autograd, clip_grad_norm_ and torch.optim.Adam.
* ``reference_shaped_train`` — the reference's own loop shape (train_gcn_dqn.py:153-178):
  B = 1, dict observations, a Python edge list rebuilt every tick, edge-list GAT,
  one coin per tick, replay as a Python list, random.sample(32) + batch concat.
"""
from __future__ import annotations

import random
import time

import numpy as np
import torch

from . import swarm_oracle as O


def _init_state(scenario, B, N, seed):
    c = O.reset_centres(scenario, B, seed, 0, shared=False)
    pos = O.grid_positions(c, N)
    return pos, torch.zeros_like(pos)


def vectorized_train(flat_params, scenario, B, N, batch, seconds=15.0, eps=0.05, seed=0, prefill=2):
    params = O.unflatten_params(flat_params)
    flat, target = flat_params.clone(), flat_params.clone()
    m = torch.zeros_like(flat)
    v = torch.zeros_like(flat)
    pos, vel = _init_state(scenario, B, N, seed)
    ring = []
    rng = np.random.default_rng(seed)
    step = 0
    ticks = 0
    t0 = None
    tick = 0
    while True:
        if ticks == prefill and t0 is None:
            t0 = time.perf_counter()
            ticks = 0
        out = O.act_tick(params, pos, vel, scenario, O.GRAPH_COMPLETE, 0, eps, seed, tick)
        ring.append((torch.cat([pos, vel], -1), out.actions, out.step["rew"],
                     torch.cat([out.step["pos"], out.step["vel"]], -1)))
        pos, vel = out.step["pos"], out.step["vel"]
        n_graphs = len(ring) * B
        if n_graphs >= batch:
            g = rng.choice(n_graphs, size=batch, replace=False)
            sl, ev = g // B, g % B
            s = torch.stack([ring[i][0][e] for i, e in zip(sl, ev)])
            a = torch.stack([ring[i][1][e] for i, e in zip(sl, ev)])
            r = torch.stack([ring[i][2][e] for i, e in zip(sl, ev)])
            s1 = torch.stack([ring[i][3][e] for i, e in zip(sl, ev)])
            res = O.td_step(flat, target, m, v, step, s, a, r, s1)
            flat, m, v, step = res["params"], res["m"], res["v"], res["step"]
            params = O.unflatten_params(flat)
        tick += 1
        ticks += 1
        if t0 is not None and time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    return dict(agent_steps_per_s=ticks * B * N / dt, ticks=ticks, seconds=dt)


def reference_shaped_train(flat_params, scenario, N, seconds=10.0, eps=0.05, seed=0, batch=32):
    random.seed(seed)
    params = O.unflatten_params(flat_params)
    flat, target = flat_params.clone(), flat_params.clone()
    m = torch.zeros_like(flat)
    v = torch.zeros_like(flat)
    pos, vel = _init_state(scenario, 1, N, seed)
    replay = []
    step = 0
    ticks = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        obs = {f"agent{i}": torch.cat([pos[:, i], vel[:, i], O.f32(O.GOAL)[None]], -1) for i in range(N)}
        x = torch.cat([torch.stack([obs[f"agent{i}"] for i in range(N)], 0).squeeze(1),
                       torch.arange(N).float().unsqueeze(1)], 1)
        ei = O.complete_edge_index(N)
        q = O.q_forward_edges(params, x, ei).detach()
        if random.random() < eps:
            acts = torch.tensor([random.randint(0, 8) for _ in range(N)])
        else:
            acts = torch.argmax(q, dim=1)
        st = O.env_step(pos, vel, acts[None], scenario)
        replay.append((torch.cat([pos, vel], -1)[0], acts, st["rew"][0], torch.cat([st["pos"], st["vel"]], -1)[0]))
        pos, vel = st["pos"], st["vel"]
        if len(replay) >= batch:
            smp = random.sample(replay, batch)
            s = torch.stack([t[0] for t in smp])
            a = torch.stack([t[1] for t in smp])
            r = torch.stack([t[2] for t in smp])
            s1 = torch.stack([t[3] for t in smp])
            res = O.td_step(flat, target, m, v, step, s, a, r, s1)
            flat, m, v, step = res["params"], res["m"], res["v"], res["step"]
            params = O.unflatten_params(flat)
        ticks += 1
    dt = time.perf_counter() - t0
    return dict(agent_steps_per_s=ticks * N / dt, ticks=ticks, seconds=dt)


def reference_shaped_eval(flat_params, scenario, N, k=5, seconds=5.0, max_steps=50, seed=0):
    """BASELINE.json configs[0] (C1): the reference's evaluation script shape
    (tests/test_go_to_position.py -> Simulator.run_simulation, simulator.py:47-109) at B = 1:
    per tick a dict of observations, the kNN edge list rebuilt with torch.topk per agent
    (simulator.py:9-26), the edge-list GAT forward under no_grad, argmax, the env step and the
    scenario metrics; episodes of ``max_steps`` ticks from the reset grid."""
    params = O.unflatten_params(flat_params)
    ticks = 0
    t0 = time.perf_counter()
    episode = 0
    while time.perf_counter() - t0 < seconds:
        pos, vel = _init_state(scenario, 1, N, seed + episode)
        for _ in range(max_steps):
            obs = {f"agent{i}": torch.cat([pos[:, i], vel[:, i], O.f32(O.GOAL)[None]], -1) for i in range(N)}
            x = torch.cat([torch.stack([obs[f"agent{i}"] for i in range(N)], 0).squeeze(1),
                           torch.arange(N).float().unsqueeze(1)], 1)
            ei = O.knn_edge_index(x[:, :2], k)
            with torch.no_grad():
                acts = torch.argmax(O.q_forward_edges(params, x, ei), dim=1)
            st = O.env_step(pos, vel, acts[None], scenario)
            _ = float(st["avg_dist"][0]), float(st["hits"][0])   # the per-tick metrics the Simulator records
            pos, vel = st["pos"], st["vel"]
            ticks += 1
        episode += 1
    dt = time.perf_counter() - t0
    return dict(agent_steps_per_s=ticks * N / dt, ticks=ticks, seconds=dt)
