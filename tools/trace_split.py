"""Where a training tick's time goes, from a rocprofv3 kernel trace of bench.py.

rocprofv3 --kernel-trace gives every dispatch a start and an end timestamp (one clock).  Summing
the kernels' durations does not reproduce the tick: under the tracer the intervals of two
consecutive dispatches of a hipGraph overlap (a dispatch's end stamp also covers its end-of-kernel
cache release, which the next dispatch's start does not wait for in full), so tick_kernel +
grad_reduce_kernel exceeded the timed tick in round 3.  This tool splits the
tick by START stamps instead, which partition the timeline exactly:

  tick share    = start(reduce of tick t) - start(tick kernel of tick t)
  reduce share  = start(tick kernel of tick t + 1) - start(reduce of tick t)

and reports beside it each kernel's traced duration, the gaps end -> next start (negative =
overlap), and the traced episode span against the sum of durations.

usage: python tools/trace_split.py gpurun_out/trace/run_kernel_trace.csv [out.json]
"""
import csv
import json
import statistics
import sys

TICK, REDUCE, RESET = "tick_kernel", "grad_reduce_kernel", "reset_kernel"


def load(path):
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def kind(name):
    for k in (TICK, REDUCE, RESET):
        if k in name:
            return k
    return "other"


def episodes(rows):
    """Runs of (tick, reduce) pairs between two resets: one bench step each."""
    eps, cur = [], []
    for st, en, name in rows:
        k = kind(name)
        if k == RESET:
            if cur:
                eps.append(cur)
            cur = []
        elif k in (TICK, REDUCE):
            cur.append((st, en, k))
        else:   # any other launch ends the run (kernel-timing chains, rollouts, ...)
            if cur:
                eps.append(cur)
            cur = []
    if cur:
        eps.append(cur)
    out = []
    for e in eps:   # keep strictly alternating tick, reduce runs
        if len(e) >= 4 and all(e[i][2] == (TICK if i % 2 == 0 else REDUCE) for i in range(len(e))):
            out.append(e)
    return out


def split(eps, ticks):
    full = [e for e in eps if len(e) == 2 * ticks]
    if not full:
        raise SystemExit(f"no episode of {ticks} (tick, reduce) pairs in the trace")
    tick_share, red_share, d_tick, d_red, gap_tr, gap_rt, spans, sums = [], [], [], [], [], [], [], []
    for e in full:
        for i in range(0, len(e), 2):
            (ts, te, _), (rs, re_, _) = e[i], e[i + 1]
            d_tick.append(te - ts)
            d_red.append(re_ - rs)
            tick_share.append(rs - ts)
            gap_tr.append(rs - te)
            if i + 2 < len(e):
                ns = e[i + 2][0]
                red_share.append(ns - rs)
                gap_rt.append(ns - re_)
        spans.append(e[-1][1] - e[0][0])
        sums.append(sum(en - st for st, en, _ in e))
    us = lambda v: round(statistics.mean(v) / 1e3, 3)
    med = lambda v: round(statistics.median(v) / 1e3, 3)
    return {
        "episodes": len(full), "ticks_per_episode": ticks,
        "tick_period_us": round(statistics.mean(spans) / ticks / 1e3, 3),
        "split_by_start_stamps_us": {"tick_kernel": us(tick_share), "grad_reduce": us(red_share)},
        "traced_duration_us": {"tick_kernel": {"mean": us(d_tick), "median": med(d_tick)},
                               "grad_reduce": {"mean": us(d_red), "median": med(d_red)}},
        "gap_end_to_next_start_us": {"tick->reduce": us(gap_tr), "reduce->tick": us(gap_rt)},
        "episode_span_vs_sum_of_durations_us": {"span": us(spans), "sum": us(sums)},
    }


def main():
    src = sys.argv[1]
    ticks = int(sys.argv[3]) if len(sys.argv) > 3 else 100
    res = split(episodes(load(src)), ticks)
    res["source"] = src
    print(json.dumps(res, indent=1))
    if len(sys.argv) > 2:
        json.dump(res, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
