#!/bin/bash
# kNN tie path rewrite: acting parity tests on the in-tree library, then the kNN acting rollout
# A/B against the legacy restatement (ab/libswarm_legacy.so)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  -k "knn or tie or rollout or recorded or act_tick or gat3 or compat or memo" > gpurun_out/tie_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/tie_tests.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/tie_tests.log | head -20; exit $rc; fi
timeout -k 10 200 python -u tools/act_waves.py 1024 8 knn 5 100 > gpurun_out/act_waves_new.log 2>&1 || exit $?
grep -E "rollout|tie-path" gpurun_out/act_waves_new.log
REPS=${REPS:-3} VARIANTS="base nomemo legacy" BENCH_ARGS="--mode act --graph knn --knn-k 5" bash scripts/ab_bench.sh > /dev/null || exit $?
cp gpurun_out/ab.jsonl gpurun_out/ab_tie_rewrite.jsonl
REPS=2 VARIANTS="base legacy" BENCH_ARGS="--mode act --graph knn --knn-k 10 --scenario ObstacleAvoidance --agents 12" bash scripts/ab_bench.sh > /dev/null || exit $?
cp gpurun_out/ab.jsonl gpurun_out/ab_tie_rewrite_oa.jsonl
python -c "
import json
for l in open('gpurun_out/ab_tie_rewrite.jsonl').readlines() + open('gpurun_out/ab_tie_rewrite_oa.jsonl').readlines():
    d = json.loads(l); print(d['variant'], d['rep'], round(d['value'] / 1e9, 3), 'G', d['ms_per_step'])"
