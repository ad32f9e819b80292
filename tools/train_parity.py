"""Statistical parity of the training path: run DQNTrainer.train_model
with the reference script's configuration (src/training/train_gcn_dqn.py:262-290: 10 agents,
1 env, 1000 episodes of 100 ticks, eps 0.99 -> 0.05 at decay 0.01, batch 32, target sync
every 200 ticks) for several seeds and compare the learning curves with the reference's
recorded ones (tests/golden/train_stats.json, from data/stats/*.csv).

The training path cannot match bit for bit (Python random / torch.randn streams and PyG's
initialisation are not reproducible), so the comparison is of distributions:
the 10-episode mean reward at checkpoints and at the end, per seed, against the reference's
10 seeds, plus Welch's t over the last-100-episode window.

The logged curve is agent 0's reward divided by the agent count (train_gcn_dqn.py:177,184).
GoTo's reward is collective (-sum of every agent's distance), so its curve does not depend on
the agent count; ObstacleAvoidance's is agent 0's own, so its curve scales as 1/N and pins
the N the recorded runs used.  ``--agents`` sweeps it.

    python tools/train_parity.py [--out out.json] [--seeds 0,1,...] [--episodes 1000]
                                 [--scenarios GoTo,ObstacleAvoidance] [--agents 10[,5,...]]
"""
import argparse
import contextlib
import io
import json
import math
import os
import statistics
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(scen_name, seed, episodes, n_agents=10):
    import swarm_amd
    scen = swarm_amd.GoToPositionScenario() if scen_name == "GoTo" else swarm_amd.ObstacleAvoidanceScenario()
    env = swarm_amd.make_env(scenario=scen, num_envs=1, continuous_actions=False, wrapper=None, max_steps=100,
                             dict_spaces=True, n_agents=n_agents, seed=seed)
    with tempfile.TemporaryDirectory() as d:
        swarm_amd.set_seed(seed)
        tr = swarm_amd.DQNTrainer(env, seed, os.path.join(d, "models"), os.path.join(d, "stats"), scen_name)
        with contextlib.redirect_stdout(io.StringIO()):
            tr.train_model({"epsilon": 0.99, "epsilon_decay": 0.01, "min_epsilon": 0.05, "episodes": episodes})
    return [float(x) for x in tr.episode_rewards]


def welch(a, b):
    """Welch's t statistic and its Welch-Satterthwaite degrees of freedom; two-sided p from
    scipy when it is importable (it is in this image), else None."""
    ma, mb = statistics.mean(a), statistics.mean(b)
    va, vb = statistics.variance(a) / len(a), statistics.variance(b) / len(b)
    t = (ma - mb) / math.sqrt(va + vb)
    df = (va + vb) ** 2 / (va ** 2 / (len(a) - 1) + vb ** 2 / (len(b) - 1))
    try:
        from scipy import stats
        p = float(2 * stats.t.sf(abs(t), df))
    except ImportError:
        p = None
    return t, df, p


def window(curve, lo, hi):
    """mean of the 10-episode means covering episodes [lo, hi)"""
    return statistics.mean(curve[lo // 10: hi // 10])


def compare(ref, scen, ours, seeds, episodes):
    k = episodes // 10 - 1                    # last 10-episode mean
    ref_c = [ref["curves"][scen][str(s)]["reward"] for s in range(10)]
    out = {"ours_final": [ours[s][k] for s in seeds], "ref_final": [c[k] for c in ref_c]}
    lo = max(0, episodes - 100)
    out["ours_last100"] = [window(ours[s], lo, episodes) for s in seeds]
    out["ref_last100"] = [window(c, lo, episodes) for c in ref_c]
    for key in ("final", "last100"):
        a, b = out[f"ours_{key}"], out[f"ref_{key}"]
        out[f"{key}_mean"] = (statistics.mean(a), statistics.mean(b))
        out[f"{key}_std"] = (statistics.stdev(a) if len(a) > 1 else 0.0, statistics.stdev(b))
        if len(a) > 1:
            t, df, p = welch(a, b)
            out[f"{key}_welch"] = {"t": t, "df": df, "p": p}
    out["checkpoints"] = {}
    for ep in (9, 99, 299, 499, 999):
        if ep < episodes:
            i = ep // 10
            out["checkpoints"][ep] = {"ours_mean": statistics.mean(ours[s][i] for s in seeds),
                                      "ref_mean": statistics.mean(c[i] for c in ref_c)}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "train_parity.json"))
    ap.add_argument("--seeds", default=",".join(str(s) for s in range(10)))
    ap.add_argument("--episodes", type=int, default=1000)
    ap.add_argument("--scenarios", default="GoTo,ObstacleAvoidance")
    ap.add_argument("--agents", default="10")
    a = ap.parse_args()
    seeds = [int(s) for s in a.seeds.split(",")]
    ref = json.load(open(os.path.join(ROOT, "tests", "golden", "train_stats.json")))
    res = {"config": ref["config"] | {"episodes": a.episodes}, "seeds": seeds, "runs": []}
    for scen in a.scenarios.split(","):
        for n in [int(x) for x in a.agents.split(",")]:
            t0 = time.time()
            ours = {s: run(scen, s, a.episodes, n) for s in seeds}
            secs = time.time() - t0
            r = compare(ref, scen, ours, seeds, a.episodes)
            r |= {"scenario": scen, "n_agents": n, "seconds": secs, "ticks": len(seeds) * a.episodes * 100,
                  "curves": {str(s): ours[s] for s in seeds}}
            res["runs"].append(r)
            w = r.get("last100_welch", {})
            print(f"{scen:18s} N={n:2d} last-100 reward: ours {r['last100_mean'][0]:8.2f} +- {r['last100_std'][0]:.2f} "
                  f"({len(seeds)} seeds)  reference {r['last100_mean'][1]:8.2f} +- {r['last100_std'][1]:.2f} "
                  f"(10 seeds)  Welch t={w.get('t', float('nan')):.2f} p={w.get('p')}  [{secs:.1f} s]", flush=True)
            fw = r.get("final_welch", {})
            print(f"    final 10-episode: ours {r['final_mean'][0]:8.2f}  reference {r['final_mean'][1]:8.2f}  "
                  f"Welch t={fw.get('t', float('nan')):.2f} p={fw.get('p')}", flush=True)
            for ep, c in r["checkpoints"].items():
                print(f"    episode {ep:4d}: ours {c['ours_mean']:8.2f}  reference {c['ref_mean']:8.2f}", flush=True)
            os.makedirs(os.path.dirname(a.out), exist_ok=True)
            json.dump(res, open(a.out, "w"))


if __name__ == "__main__":
    main()
