"""``Simulator`` — the reference's scalability-evaluation loop (src/simulation/simulator.py:28-166)
on the device: per episode one ``swarm_rollout`` launch runs ``max_steps`` ticks of
kNN graph -> GAT -> argmax -> env.step with frozen weights and records per-tick
positions, average distance and hits; the CSV outputs keep the reference's
layout (``result.csv``, ``positions/positions_episode_{e}_{x,y}.csv``,
``data/distances_episode_{e}.csv``).  ``knn_k`` defaults to the code's 10; the
reference's committed outputs were produced with 5.  ``graph="radius"`` with
``radius=r`` evaluates on the north_star's radius-neighbour graph instead (not in the
reference).
With ``num_envs`` > 1, metrics are averaged over envs and trajectories of env 0
are written.
"""
from __future__ import annotations

import csv
import ctypes
import os
import time

import torch

from . import _lib


class Simulator:
    def __init__(self, env, model, episodes, env_name, seed, output_dir="test_stats/", render=False, knn_k: int = 10,
                 graph: str = "knn", radius: float = 0.3):
        self.env = env
        self.model = model
        self.episode_rewards = []
        self.distance_at_the_end = []
        self.distance_at_the_beginning = []
        self.total_collisions = []
        self.episodes = episodes
        self.env_name = env_name
        self.seed = seed
        self.output_dir = output_dir
        self.render = render
        self.knn_k = knn_k
        if graph not in ("knn", "radius"):
            raise ValueError("graph must be 'knn' (simulator.py:15-24) or 'radius'")
        self.graph = _lib.GRAPH_KNN if graph == "knn" else _lib.GRAPH_RADIUS
        self.radius = float(radius)
        self.all_positions_x = []
        self.all_positions_y = []
        self.all_distances = []
        self.all_hits = []

    def run_simulation(self):
        if self.graph == _lib.GRAPH_KNN and self.knn_k > self.env.n_agents:
            raise RuntimeError("selected index k out of range")
        eng = self.env.engine
        params = self.model.flat_params(eng.device)
        conv = _lib.CONV_GAT if getattr(self.model, "conv", "gat") == "gat" else _lib.CONV_GCN
        saved = (eng.cfg.graph, eng.cfg.knn_k, eng.cfg.conv, eng.cfg.radius, eng.cfg.net)
        eng.cfg.graph, eng.cfg.knn_k, eng.cfg.conv, eng.cfg.radius = self.graph, self.knn_k, conv, self.radius
        eng.cfg.net = getattr(self.model, "net_id", _lib.NET_GCN)   # the Flocking checkpoints' GAT3
        T = self.env.max_steps
        try:
            for episode in range(self.episodes):
                self.env.reset()
                t0 = time.time()
                res = eng.rollout(T, tick0=episode * T, eps=0.0, traj=True, params=params)
                pos = res["traj_pos"][:, 0].cpu()            # [T, N, 2] env 0
                dist = res["traj_dist"].mean(dim=1).cpu()     # [T]
                hits = res["traj_hits"].mean(dim=1).cpu()
                total_reward = res["reward"].sum(dim=1).mean()
                self.all_positions_x.append(pos[:, :, 0].tolist())
                self.all_positions_y.append(pos[:, :, 1].tolist())
                self.all_distances.append(dist.tolist())
                self.all_hits.append(hits.tolist())
                print(f"It took: {time.time() - t0}s for {T} steps of episode {episode} with "
                      f"{float(total_reward)} total reward, on device {eng.device} for test_gcn_vmas scenario.")
                self.total_collisions.append(hits.sum())
                self.distance_at_the_end.append(dist[-1])
                self.distance_at_the_beginning.append(dist[0])
                self.episode_rewards.append(float(total_reward) / T)
        finally:
            eng.cfg.graph, eng.cfg.knn_k, eng.cfg.conv, eng.cfg.radius, eng.cfg.net = saved
        self.save_metrics_to_csv()

    def save_metrics_to_csv(self):
        where = self.output_dir
        os.makedirs(where, exist_ok=True)
        with open(where + "/result.csv", mode="w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Episode", "Reward", "Collisions", "Distance (end)", "Distance (beginning)"])
            for i in range(self.episodes):
                w.writerow([i, self.episode_rewards[i], float(self.total_collisions[i]),
                            float(self.distance_at_the_end[i]), float(self.distance_at_the_beginning[i])])
        pdir = f"{where}/positions"
        os.makedirs(pdir, exist_ok=True)
        for axis, allp in (("x", self.all_positions_x), ("y", self.all_positions_y)):
            for i, ep in enumerate(allp):
                with open(f"{pdir}/positions_episode_{i}_{axis}.csv", mode="w", newline="") as f:
                    w = csv.writer(f)
                    w.writerow(["Tick"] + [f"{axis.upper()}{j}" for j in range(len(ep[0]))])
                    for j, row in enumerate(ep):
                        w.writerow([j] + row)
        ddir = f"{where}/data"
        os.makedirs(ddir, exist_ok=True)
        for i in range(len(self.all_distances)):
            with open(f"{ddir}/distances_episode_{i}.csv", mode="w", newline="") as f:
                w = csv.writer(f)
                w.writerow(["Tick", "Distance", "Hits"])
                for j in range(len(self.all_distances[i])):
                    w.writerow([j, self.all_distances[i][j], self.all_hits[i][j]])
