#!/bin/bash
# Round 6 verification (call B): the PMC passes at C3 and C5's N = 12 shard (scripts/r05_counters.sh),
# the PMC passes of the acting line's kNN-5 rollout (bench.py --mode act), summarised with the build
# identity, then the 40-step headline line and the sweep of every BASELINE configuration
# (scripts/sweep.sh).  Stops at the first failure.
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/r05_counters.sh || exit $?
OUT=gpurun_out/pmc_act BENCH_ARGS="--mode act --graph knn --knn-k 5 --steps 3 --warmup 1 --no-kernel-timing" bash scripts/pmc.sh || exit $?
python tools/pmc_summary.py gpurun_out/pmc_act gpurun_out/pmc_rollout.json || exit $?
bash scripts/sweep.sh || exit $?
echo "final B ok"
