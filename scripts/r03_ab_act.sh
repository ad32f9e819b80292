#!/bin/bash
# acting-only kNN rollout A/B (tie-path code layout, rollout occupancy target), gated by the
# acting parity tests of each variant
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in $VARIANTS; do
  [ "$v" = base ] && continue
  SWARM_LIB_PATH=$PWD/ab/libswarm_$v.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
    -k "knn or rollout or recorded or act_tick or gat3" > gpurun_out/ab_tests_$v.log 2>&1
  rc=$?; echo "variant $v tests rc=$rc"; tail -1 gpurun_out/ab_tests_$v.log
  if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/ab_tests_$v.log | head -20; exit $rc; fi
done
REPS=${REPS:-3} BENCH_ARGS="--mode act --graph knn --knn-k 5" bash scripts/ab_bench.sh > /dev/null || exit $?
cp gpurun_out/ab.jsonl gpurun_out/ab_act_knn.jsonl
REPS=2 BENCH_ARGS="--mode act" bash scripts/ab_bench.sh > /dev/null || exit $?
cp gpurun_out/ab.jsonl gpurun_out/ab_act_complete.jsonl
cat gpurun_out/ab_act_knn.jsonl gpurun_out/ab_act_complete.jsonl | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['variant'], d['rep'], round(d['value'] / 1e9, 3), 'G', d['ms_per_step'])"
