#!/bin/bash
# kNN acting-only A/B (tie path out of line / skipped) and the hand-off poll without sleep
export TMPDIR=/tmp
mkdir -p gpurun_out
SWARM_LIB_PATH=$PWD/ab/libswarm_tieni.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  -k "knn or rollout or recorded or act_tick" > gpurun_out/ab_tests_tieni.log 2>&1
rc=$?; echo "tieni tests rc=$rc"; tail -2 gpurun_out/ab_tests_tieni.log
if [ $rc -ne 0 ]; then exit $rc; fi
VARIANTS="base tieni notie" REPS=3 BENCH_ARGS="--mode act --graph knn --knn-k 5" bash scripts/ab_bench.sh > /dev/null || exit $?
cp gpurun_out/ab.jsonl gpurun_out/ab_knn.jsonl
VARIANTS="base hs0" bash scripts/ab_check.sh > /dev/null || exit $?
cat gpurun_out/ab_knn.jsonl gpurun_out/ab.jsonl
