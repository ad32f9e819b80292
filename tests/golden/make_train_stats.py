"""Extract the reference's recorded training curves into a small fixture.

Run in the build container (``/root/reference`` is read-only and absent on the GPU box):
``python tests/golden/make_train_stats.py``.

Source: ``data/stats/experiment_{GoTo,ObstacleAvoidance}-seed_{0..9}.csv``, written by
``DQNTrainer.save_metrics_to_csv`` (``src/training/train_gcn_dqn.py:225-231``) after
``train_model`` with the script's config (``:262-290``: 10 agents, 1 env, 1000 episodes of
100 ticks, ε 0.99 -> 0.05 at decay 0.01, batch 32, target sync every 200 ticks).  Each row
is (episode i, mean over episodes i-9..i of the per-episode reward, a loss value); the
Reward column is what the statistical parity of the training path is checked against.
No reference code is executed; only the CSV files are read.
"""
import csv
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/data/stats"


def main():
    out = {"source": "data/stats/experiment_*-seed_*.csv (reference training runs)",
           "config": {"n_agents": 10, "num_envs": 1, "episodes": 1000, "max_steps": 100, "epsilon": 0.99,
                      "epsilon_decay": 0.01, "min_epsilon": 0.05, "batch": 32, "update_target_every": 200},
           "curves": {}}
    for scen in ("GoTo", "ObstacleAvoidance"):
        out["curves"][scen] = {}
        for seed in range(10):
            rows = list(csv.reader(open(f"{REF}/experiment_{scen}-seed_{seed}.csv")))[1:]
            out["curves"][scen][str(seed)] = {"episode": [int(r[0]) for r in rows],
                                              "reward": [float(r[1]) for r in rows]}
    json.dump(out, open(os.path.join(HERE, "train_stats.json"), "w"))


if __name__ == "__main__":
    main()
