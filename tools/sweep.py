"""Bench lines for the BASELINE.json configs beside the headline (C3, the per-GPU share of C5, and
acting-only rollouts), one bench.py subprocess each, appended to a JSON-lines file.

    python tools/sweep.py [out.jsonl] [substring filter on the run names]
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "sweep.jsonl")
COMMON = ["--no-cpu-baseline", "--steps", "20", "--warmup", "3"]

RUNS = [("C3 OA 12x1024 GAT train", ["--scenario", "ObstacleAvoidance", "--agents", "12"])]
# C5 per GPU: 4096 envs over 8 GPUs = 512 envs/GPU, N = 5..12, GCN vs GAT
for conv in ("gat", "gcn"):
    for n in range(5, 13):
        RUNS.append((f"C5 OA {n}x512 {conv.upper()} train",
                     ["--scenario", "ObstacleAvoidance", "--agents", str(n), "--envs", "512", "--conv", conv]))
RUNS += [
    ("C2 GoTo 8x1024 GCN train", ["--conv", "gcn"]),
    # also the reference's absolute TD batch, S = 32 graphs per tick
    ("C2 GoTo 8x1024 GAT train S=32", ["--batch", "32"]),
    ("C2 GoTo 8x1024 GAT act kNN-5", ["--mode", "act", "--graph", "knn", "--knn-k", "5"]),
    ("C2 GoTo 8x1024 GAT act complete", ["--mode", "act"]),
    ("C3 OA 12x1024 GAT act kNN-10", ["--mode", "act", "--scenario", "ObstacleAvoidance", "--agents", "12",
                                      "--graph", "knn", "--knn-k", "10"]),
    # the north_star's radius-neighbour graph (not in the reference; fused tick, radius + GAT specialised)
    ("C2 GoTo 8x1024 GAT act radius-0.3", ["--mode", "act", "--graph", "radius", "--radius", "0.3"]),
    ("C2 GoTo 8x1024 GAT train radius-0.3", ["--graph", "radius", "--radius", "0.3"]),
    # the Flocking scenario (one-layer GCN training, as train_model('Flocking'))
    # and the Flocking checkpoints' three-layer GAT acting
    ("Flocking 8x1024 GAT train", ["--scenario", "Flocking"]),
    ("Flocking 8x1024 GAT3 act kNN-5", ["--scenario", "Flocking", "--mode", "act", "--net", "gat3",
                                        "--graph", "knn", "--knn-k", "5"]),
    ("Flocking 8x1024 GAT3 act complete", ["--scenario", "Flocking", "--mode", "act", "--net", "gat3"]),
]

if len(sys.argv) > 2:
    RUNS = [r for r in RUNS if sys.argv[2] in r[0]]
os.makedirs(os.path.dirname(OUT), exist_ok=True)
with open(OUT, "w") as f:
    for name, extra in RUNS:
        cmd = [sys.executable, os.path.join(ROOT, "bench.py")] + COMMON + extra
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=240)
        if p.returncode != 0:
            print(f"{name}: rc={p.returncode}\n{p.stderr[-2000:]}", flush=True)
            sys.exit(p.returncode)
        line = json.loads(p.stdout.strip().splitlines()[-1])
        line["sweep"] = name
        f.write(json.dumps(line) + "\n")
        f.flush()
        r = line.get("roofline") or {}
        tick_us = line.get("us_per_tick") or line["ms_per_step"] * 10   # acting: 100-tick episodes
        print(f"{name:40s} {line['value'] / 1e6:9.1f} M agent-steps/s  {tick_us:7.2f} us/tick  "
              f"frac={r.get('frac', float('nan')):.4f}", flush=True)
