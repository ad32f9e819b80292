"""Interleaved A/B of whole source trees on one GPU box.

Each variant is a directory holding a complete checkout with its own built library: "." (this
tree) or abx/<name> (a `git worktree` of another commit, built there with its build.py).  Every
round runs `python bench.py <args>` once per variant, in turn, each as a child process under its
own time limit, and appends one JSON line per run to the output file: the variant, the round,
the whole-step rate, the per-tick spread and the per-kernel chain periods of the bench line.

usage: python tools/ab_trees.py OUT.jsonl ROUNDS VARIANT[,VARIANT...] [bench args...]
       e.g. python tools/ab_trees.py gpurun_out/ab.jsonl 3 abx/base,. --steps 40 --no-cpu-baseline
"""
import json
import os
import subprocess
import sys
import time


def run(variant: str, args, timeout: int = 420) -> dict:
    cwd = os.path.abspath(variant)
    os.makedirs(os.path.join(cwd, "profiles"), exist_ok=True)   # abx trees travel without theirs
    t0 = time.time()
    p = subprocess.run([sys.executable, "bench.py", *args], cwd=cwd, capture_output=True, text=True, timeout=timeout)
    if p.returncode != 0:
        raise SystemExit(f"{variant}: bench.py exited {p.returncode}\n{p.stderr[-3000:]}")
    line = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    roof = line.get("roofline") or {}
    return {"variant": variant, "us_per_tick": line["us_per_tick"], "tick_us": line.get("tick_us"),
            "value": line["value"], "kernel_us": roof.get("kernel_us"), "frac": roof.get("frac"),
            "workload": line["config"]["workload"], "build": line.get("build", {}).get("info"),
            "wall_s": round(time.time() - t0, 1)}


def main():
    out, rounds, variants = sys.argv[1], int(sys.argv[2]), sys.argv[3].split(",")
    args = sys.argv[4:]
    with open(out, "a") as f:
        for r in range(rounds):
            for v in variants:
                rec = run(v, args)
                rec["round"] = r
                f.write(json.dumps(rec) + "\n")
                f.flush()
                print(f"round {r} {v:12s} {rec['us_per_tick']:8.3f} us/tick  tick kernel "
                      f"{(rec['kernel_us'] or {}).get('tick_kernel')}", flush=True)


if __name__ == "__main__":
    main()
