#!/bin/bash
# Round 5: the PMC passes (scripts/pmc.sh) of the final build at C3 (OA 12 x 1024) and C5's N = 12
# shard (OA 12 x 512), summarised per dispatch (tools/pmc_summary.py)
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/pmc_c3 BENCH_ARGS="--steps 5 --warmup 1 --no-cpu-baseline --no-kernel-timing --scenario ObstacleAvoidance --agents 12" bash scripts/pmc.sh || exit $?
python tools/pmc_summary.py gpurun_out/pmc_c3 gpurun_out/counters_c3.json || exit $?
OUT=gpurun_out/pmc_c5 BENCH_ARGS="--steps 5 --warmup 1 --no-cpu-baseline --no-kernel-timing --scenario ObstacleAvoidance --agents 12 --envs 512" bash scripts/pmc.sh || exit $?
python tools/pmc_summary.py gpurun_out/pmc_c5 gpurun_out/counters_c5_n12.json || exit $?
echo "counters ok"
