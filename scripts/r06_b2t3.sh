#!/bin/bash
# Round 6: write-through B2-tile stores (b2tsc1) vs all slab stores write-through (b2tall): bit for bit
# against the in-tree library, then the interleaved A/B at C2, C3, C5 N = 12 and C5 N = 5.
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/r06_bitcmp3.jsonl
for v in b2tsc1 b2tall; do
  for cfg in "GoTo 8 1024 6" "ObstacleAvoidance 12 1024 4" "ObstacleAvoidance 5 512 4"; do
    timeout -k 10 300 python tools/bitcmp.py base ab/libswarm_$v.so $cfg >> gpurun_out/r06_bitcmp3.jsonl 2> gpurun_out/r06_bitcmp3.err || { tail -5 gpurun_out/r06_bitcmp3.err; exit 1; }
  done
done
python -c "
import json
for l in open('gpurun_out/r06_bitcmp3.jsonl'):
    d = json.loads(l); print(d['b'], d['config'], d['all_bitwise'], d['grad_max_abs_diff'])
"
TAG=b2t3 V="base b2tsc1 b2tall" V3="base b2tsc1 b2tall" V5="base b2tsc1 b2tall" bash scripts/r06_ab.sh || exit $?
VARIANTS="base b2tsc1 b2tall" REPS=2 BENCH_ARGS="--steps 10 --scenario ObstacleAvoidance --agents 5 --envs 512" bash scripts/ab_bench.sh > gpurun_out/r06_b2t3_c5n5.log 2>&1 || exit 1
cp gpurun_out/ab.jsonl gpurun_out/r06_b2t3_c5n5.jsonl
echo done
