#!/bin/bash
# Round 6 interleaved A/B of library variants (tools/ab_build.py -> ab/libswarm_<name>.so; "base" =
# the in-tree library): $V at C2 ($REPS rounds), $V3 at C3 and $V5 at C5's N = 12 shard (2 rounds
# each, when set).  Output: gpurun_out/r06_<TAG>_{c2,c3,c5}.jsonl.  Stops at the first failure.
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-ab}
VARIANTS="$V" REPS=${REPS:-3} BENCH_ARGS="--steps 20" bash scripts/ab_bench.sh > gpurun_out/r06_${TAG}_c2.log 2>&1 || { tail -20 gpurun_out/r06_${TAG}_c2.log; exit 1; }
cp gpurun_out/ab.jsonl gpurun_out/r06_${TAG}_c2.jsonl
if [ -n "$V3" ]; then
VARIANTS="$V3" REPS=2 BENCH_ARGS="--steps 10 --scenario ObstacleAvoidance --agents 12" bash scripts/ab_bench.sh > gpurun_out/r06_${TAG}_c3.log 2>&1 || { tail -20 gpurun_out/r06_${TAG}_c3.log; exit 1; }
cp gpurun_out/ab.jsonl gpurun_out/r06_${TAG}_c3.jsonl
fi
if [ -n "$V5" ]; then
VARIANTS="$V5" REPS=2 BENCH_ARGS="--steps 10 --scenario ObstacleAvoidance --agents 12 --envs 512" bash scripts/ab_bench.sh > gpurun_out/r06_${TAG}_c5.log 2>&1 || { tail -20 gpurun_out/r06_${TAG}_c5.log; exit 1; }
cp gpurun_out/ab.jsonl gpurun_out/r06_${TAG}_c5.jsonl
fi
echo "ab ok"
