"""Statistical parity of the training path: run DQNTrainer.train_model
with the reference script's configuration (src/training/train_gcn_dqn.py:262-290: 10 agents,
1 env, 1000 episodes of 100 ticks, eps 0.99 -> 0.05 at decay 0.01, batch 32, target sync
every 200 ticks) for several seeds and compare the learning curves with the reference's
recorded ones (tests/golden/train_stats.json, from data/stats/*.csv).

The training path cannot match bit for bit (Python random / torch.randn streams and PyG's
initialisation are not reproducible), so the comparison is of distributions:
the 10-episode mean reward at checkpoints and at the end, per seed, against the reference's
10 seeds.

    python tools/train_parity.py [out.json] [seeds (default 0-9)] [episodes (default 1000)]
"""
import contextlib
import io
import json
import os
import statistics
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(scen_name, seed, episodes):
    import swarm_amd
    scen = swarm_amd.GoToPositionScenario() if scen_name == "GoTo" else swarm_amd.ObstacleAvoidanceScenario()
    env = swarm_amd.make_env(scenario=scen, num_envs=1, continuous_actions=False, wrapper=None, max_steps=100,
                             dict_spaces=True, n_agents=10, seed=seed)
    with tempfile.TemporaryDirectory() as d:
        swarm_amd.set_seed(seed)
        tr = swarm_amd.DQNTrainer(env, seed, os.path.join(d, "models"), os.path.join(d, "stats"), scen_name)
        with contextlib.redirect_stdout(io.StringIO()):
            tr.train_model({"epsilon": 0.99, "epsilon_decay": 0.01, "min_epsilon": 0.05, "episodes": episodes})
    return [float(x) for x in tr.episode_rewards]


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "train_parity.json")
    seeds = [int(s) for s in sys.argv[2].split(",")] if len(sys.argv) > 2 else list(range(10))
    episodes = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
    ref = json.load(open(os.path.join(ROOT, "tests", "golden", "train_stats.json")))
    res = {"config": ref["config"] | {"episodes": episodes}, "seeds": seeds, "scenarios": {}}
    for scen in ("GoTo", "ObstacleAvoidance"):
        t0 = time.time()
        ours = {s: run(scen, s, episodes) for s in seeds}
        secs = time.time() - t0
        k = episodes // 10 - 1                    # last 10-episode mean
        ref_fin = [ref["curves"][scen][str(s)]["reward"][k] for s in range(10)]
        our_fin = [ours[s][k] for s in seeds]
        checkpoints = {}
        for ep in (99, 299, 499, 999):
            if ep < episodes:
                i = ep // 10
                checkpoints[ep] = {"ours_mean": statistics.mean(ours[s][i] for s in seeds),
                                   "ref_mean": statistics.mean(ref["curves"][scen][str(s)]["reward"][i] for s in range(10))}
        res["scenarios"][scen] = {
            "ours_final": our_fin, "ref_final": ref_fin,
            "ours_mean": statistics.mean(our_fin), "ours_std": statistics.pstdev(our_fin),
            "ref_mean": statistics.mean(ref_fin), "ref_std": statistics.stdev(ref_fin),
            "checkpoints": checkpoints, "seconds": secs, "ticks": len(seeds) * episodes * 100,
            "curves": {str(s): ours[s] for s in seeds}}
        r = res["scenarios"][scen]
        print(f"{scen:18s} final 10-episode reward: ours {r['ours_mean']:8.2f} +- {r['ours_std']:.2f} "
              f"({len(seeds)} seeds)  reference {r['ref_mean']:8.2f} +- {r['ref_std']:.2f} (10 seeds)  "
              f"[{secs:.1f} s, {r['ticks']} ticks]", flush=True)
        for ep, c in checkpoints.items():
            print(f"    episode {ep:4d}: ours {c['ours_mean']:8.2f}  reference {c['ref_mean']:8.2f}", flush=True)
    os.makedirs(os.path.dirname(out_path), exist_ok=True)
    json.dump(res, open(out_path, "w"))


if __name__ == "__main__":
    main()
