#!/bin/bash
# Round 6: write-through B2-tile stores (b2tsc1) with and without the acting replay / state stores
# write-through too (b2tsc1aw): bit for bit against the in-tree library, then the interleaved A/B.
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/r06_bitcmp4.jsonl
for cfg in "GoTo 8 1024 6" "ObstacleAvoidance 12 1024 4" "ObstacleAvoidance 5 512 4"; do
  timeout -k 10 300 python tools/bitcmp.py base ab/libswarm_b2tsc1aw.so $cfg >> gpurun_out/r06_bitcmp4.jsonl 2> gpurun_out/r06_bitcmp4.err || { tail -5 gpurun_out/r06_bitcmp4.err; exit 1; }
done
python -c "
import json
for l in open('gpurun_out/r06_bitcmp4.jsonl'):
    d = json.loads(l); print(d['b'], d['config'], d['all_bitwise'], d['grad_max_abs_diff'])
"
TAG=aw V="base b2tsc1 b2tsc1aw" V3="base b2tsc1 b2tsc1aw" V5="base b2tsc1 b2tsc1aw" REPS=4 bash scripts/r06_ab.sh || exit $?
VARIANTS="base b2tsc1 b2tsc1aw" REPS=2 BENCH_ARGS="--steps 10 --scenario ObstacleAvoidance --agents 5 --envs 512" bash scripts/ab_bench.sh > gpurun_out/r06_aw_c5n5.log 2>&1 || exit 1
cp gpurun_out/ab.jsonl gpurun_out/r06_aw_c5n5.jsonl
python tools/ab_summary.py gpurun_out/r06_aw_c2.jsonl gpurun_out/r06_aw_c3.jsonl gpurun_out/r06_aw_c5.jsonl gpurun_out/r06_aw_c5n5.jsonl
