"""Extract the reference's recorded evaluation summaries into a small fixture.

Run in the build container (``/root/reference`` is read-only and absent on the GPU box):
``python tests/golden/make_eval_stats.py``.

Source: ``data/test_stats/{go_to,obstacle_avoidance}/seed_{0..9}/agents_{5..12}/result.csv``,
written by ``Simulator.save_metrics_to_csv`` (``src/simulation/simulator.py:111-166``) when
``tests/test_go_to_position.py`` / ``tests/test_obstacle_avoidance.py`` ran the trained models
(8 episodes, GoTo 50 ticks, ObstacleAvoidance 100 ticks, random starts, kNN k = 5).  Rows:
Episode, Reward, Collisions, Distance (end), Distance (beginning).  Only CSV files are read.
"""
import csv
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/data/test_stats"


def main():
    out = {"source": "data/test_stats/*/seed_*/agents_*/result.csv (reference evaluation runs)",
           "columns": ["reward", "collisions", "distance_end", "distance_begin"], "results": {}}
    for scen in ("go_to", "obstacle_avoidance"):
        out["results"][scen] = {}
        for seed in range(10):
            for n in range(5, 13):
                rows = list(csv.reader(open(f"{REF}/{scen}/seed_{seed}/agents_{n}/result.csv")))[1:]
                out["results"][scen][f"{seed}/{n}"] = [[float(v) for v in r[1:5]] for r in rows]
    json.dump(out, open(os.path.join(HERE, "eval_stats.json"), "w"))


if __name__ == "__main__":
    main()
