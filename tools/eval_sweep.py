"""The reference's evaluation harness (tests/test_go_to_position.py, tests/test_obstacle_avoidance.py
-> Simulator, src/simulation/simulator.py) on the device, over the recorded grid: model seeds
0-9 x agents 5-12 x 8 episodes, GoTo 50 ticks / ObstacleAvoidance 100 ticks, random starts,
kNN k = 5 (the recorded data's k).  Writes the reference's CSV layout
(<out>/<scenario>/seed_<s>/agents_<n>/{result.csv, positions/, data/}) and compares the
per-(scenario, agents) means of Reward, Collisions and Distance (end) with the reference's
recorded result.csv files (tests/golden/eval_stats.json).  Start positions come from Philox,
not torch.randn, so the comparison is of distributions (the policies themselves are pinned
tick by tick by tests/test_gpu_parity.py::test_gpu_reproduces_recorded_reference_actions).

    python tools/eval_sweep.py [out_dir] [seeds (default 0-9)] [agents (default 5-12)]
"""
import contextlib
import io
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SCEN = {"go_to": ("GoToPositionScenario", "weights_go_to", 50),
        "obstacle_avoidance": ("ObstacleAvoidanceScenario", "weights_obstacle_avoidance", 100),
        # the Flocking checkpoints (three GATConvs, hidden 8): the reference records no
        # Flocking evaluation, so these rows have no reference column (parity unpinned)
        "flocking": ("FlockingScenario", "weights_flocking", 100)}


def run_one(scen, seed, n, out_dir, weights):
    import swarm_amd
    from oracle import swarm_oracle as O
    cls, wkey, T = SCEN[scen]
    env = swarm_amd.make_env(getattr(swarm_amd, cls)(), scenario_name="test_gcn_vmas", num_envs=1,
                             continuous_actions=False, dict_spaces=True, wrapper=None, seed=6967, n_agents=n,
                             max_steps=T, random=True)
    if scen == "flocking":
        model = swarm_amd.GCN.from_state_dict(O.gat3_unflatten(torch.tensor(weights[wkey][seed])))
    else:
        model = swarm_amd.GCN(7, 32, 9)
        model.load_state_dict(O.unflatten_params(torch.tensor(weights[wkey][seed])))
    d = os.path.join(out_dir, scen, f"seed_{seed}", f"agents_{n}")
    sim = swarm_amd.Simulator(env, model, 8, scen, 6967, output_dir=d, knn_k=5)
    with contextlib.redirect_stdout(io.StringIO()):
        sim.run_simulation()
    rows = np.loadtxt(os.path.join(d, "result.csv"), delimiter=",", skiprows=1, ndmin=2)
    return rows[:, 1:5].tolist()


def main():
    out_dir = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "eval_sweep")
    seeds = [int(s) for s in sys.argv[2].split(",")] if len(sys.argv) > 2 else list(range(10))
    agents = [int(s) for s in sys.argv[3].split(",")] if len(sys.argv) > 3 else list(range(5, 13))
    weights = dict(np.load(os.path.join(ROOT, "tests", "golden", "weights.npz")))
    weights.update(np.load(os.path.join(ROOT, "tests", "golden", "flocking_weights.npz")))
    only = os.environ.get("EVAL_SCENARIOS")   # e.g. "flocking"
    scens = [x for x in SCEN if not only or x in only.split(",")]
    ref = json.load(open(os.path.join(ROOT, "tests", "golden", "eval_stats.json")))["results"]
    summary = {"seeds": seeds, "agents": agents, "episodes": 8, "rows": {}}
    for scen in scens:
        t0 = time.time()
        print(f"{scen}: mean over {len(seeds)} seeds x 8 episodes (ours | reference)", flush=True)
        print("  agents   reward              collisions        distance(end)     distance(begin)", flush=True)
        for n in agents:
            ours = [r for s in seeds for r in run_one(scen, s, n, out_dir, weights)]
            theirs = [r for s in range(10) for r in ref[scen][f"{s}/{n}"]] if scen in ref else None
            row = {}
            for j, name in enumerate(("reward", "collisions", "distance_end", "distance_begin")):
                a = [r[j] for r in ours]
                b = [r[j] for r in theirs] if theirs else [float("nan")]
                row[name] = {"ours_mean": statistics.mean(a), "ours_std": statistics.pstdev(a),
                             "ref_mean": statistics.mean(b), "ref_std": statistics.pstdev(b) if theirs else None}
            summary["rows"][f"{scen}/{n}"] = row
            print(f"  {n:6d}   " + "   ".join(f"{row[k]['ours_mean']:7.3f} | {row[k]['ref_mean']:7.3f}"
                                             for k in ("reward", "collisions", "distance_end", "distance_begin")),
                  flush=True)
        print(f"  [{time.time() - t0:.1f} s]", flush=True)
    json.dump(summary, open(os.path.join(out_dir, "summary.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
