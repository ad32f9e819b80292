#!/bin/bash
# Round 6: the slab's remaining pieces as 16-B write-through stores in the blocks holding none of this
# tick's transitions only (SWARM_WT_REST=2): bit for bit against the in-tree library, then the A/B.
# NOTE: the SWARM_WT_REST=2 sources are scripts/patches/r06_wtrest2.patch (git apply, then tools/ab_build.py
# wtrest2=-DSWARM_WT_REST=2); the knob is not in the tree, so without the patch the variant is the product library.
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/r06_bitcmp6.jsonl
for cfg in "GoTo 8 1024 6" "ObstacleAvoidance 12 1024 4" "ObstacleAvoidance 5 512 4" "ObstacleAvoidance 12 512 4" "GoTo 8 64 8"; do
  timeout -k 10 300 python tools/bitcmp.py base ab/libswarm_wtrest2.so $cfg >> gpurun_out/r06_bitcmp6.jsonl 2> gpurun_out/r06_bitcmp6.err || { tail -5 gpurun_out/r06_bitcmp6.err; exit 1; }
done
python -c "
import json
for l in open('gpurun_out/r06_bitcmp6.jsonl'):
    d = json.loads(l); print(d['b'], d['config'], d['all_bitwise'], d['grad_max_abs_diff'])
"
TAG=wtrest2 V="base wtrest2" V3="base wtrest2" V5="base wtrest2" REPS=4 bash scripts/r06_ab.sh || exit $?
VARIANTS="base wtrest2" REPS=2 BENCH_ARGS="--steps 10 --scenario ObstacleAvoidance --agents 5 --envs 512" bash scripts/ab_bench.sh > gpurun_out/r06_wtrest2_c5n5.log 2>&1 || exit 1
cp gpurun_out/ab.jsonl gpurun_out/r06_wtrest2_c5n5.jsonl
python tools/ab_summary.py gpurun_out/r06_wtrest2_c2.jsonl gpurun_out/r06_wtrest2_c3.jsonl gpurun_out/r06_wtrest2_c5.jsonl gpurun_out/r06_wtrest2_c5n5.jsonl
