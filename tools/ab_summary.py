"""Print an A/B jsonl (scripts/ab_bench.sh) as per-variant means: us per tick, the tick kernel's
chain period and the tick period.  usage: python tools/ab_summary.py FILE.jsonl [...]"""
import collections
import json
import sys

for f in sys.argv[1:]:
    agg = collections.defaultdict(list)
    for line in open(f):
        d = json.loads(line)
        k = d.get("kernel_us") or {}
        agg[d["variant"]].append((d["us_per_tick"], k.get("tick_kernel") or 0.0, k.get("tick_period (tick + reduce)") or 0.0))
    base = None
    for v, x in agg.items():
        m = [sum(c) / len(c) for c in zip(*x)]
        base = m if base is None else base
        print(f"{f.split('/')[-1]:28s} {v:12s} n={len(x)}  us/tick {m[0]:7.3f} ({m[0] - base[0]:+.3f})  "
              f"tick kernel {m[1]:6.2f}  tick period {m[2]:6.2f}")
