#!/bin/bash
# GPU suite, then interleaved A/B of the in-tree library (base) against ab/libswarm_old.so at C2
# and C3, then the stamps timeline of the in-tree code.  Stops at the first failure.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/pytest_gpu.log | head -30; exit $rc; fi
VARIANTS="${VARIANTS:-base old}" REPS=${REPS:-3} bash scripts/ab_bench.sh > /dev/null || exit $?
cp gpurun_out/ab.jsonl gpurun_out/ab_c2.jsonl; cat gpurun_out/ab_c2.jsonl | cut -c1-200
VARIANTS="${VARIANTS:-base old}" REPS=2 BENCH_ARGS="--scenario ObstacleAvoidance --agents 12" bash scripts/ab_bench.sh > /dev/null || exit $?
cp gpurun_out/ab.jsonl gpurun_out/ab_c3.jsonl; cat gpurun_out/ab_c3.jsonl | cut -c1-200
if [ -n "$TIMELINE" ]; then
  timeout -k 10 300 python tools/tick_timeline.py > gpurun_out/timeline.txt 2>&1 || exit $?
  grep -E "tick|without|slowest" gpurun_out/timeline.txt
fi
