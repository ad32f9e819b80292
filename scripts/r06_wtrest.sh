#!/bin/bash
# Round 6: the slab's remaining pieces (vector sums by DPP lane gathers, dW rows through LDS) as 16-B
# write-through stores too (SWARM_WT_REST): bit for bit against the in-tree library, then the A/B.
# NOTE: the SWARM_WT_REST knob was removed after this A/B (ce97a8a); its sources are at 6f7b431, so rebuilding the variants from today's tree builds the product library.
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/r06_bitcmp5.jsonl
for cfg in "GoTo 8 1024 6" "ObstacleAvoidance 12 1024 4" "ObstacleAvoidance 5 512 4" "ObstacleAvoidance 12 512 4" "GoTo 8 64 8"; do
  timeout -k 10 300 python tools/bitcmp.py base ab/libswarm_wtrest.so $cfg >> gpurun_out/r06_bitcmp5.jsonl 2> gpurun_out/r06_bitcmp5.err || { tail -5 gpurun_out/r06_bitcmp5.err; exit 1; }
done
python -c "
import json
for l in open('gpurun_out/r06_bitcmp5.jsonl'):
    d = json.loads(l); print(d['b'], d['config'], d['all_bitwise'], d['grad_max_abs_diff'])
"
TAG=wtrest V="base wtrest" V3="base wtrest" V5="base wtrest" REPS=4 bash scripts/r06_ab.sh || exit $?
VARIANTS="base wtrest" REPS=2 BENCH_ARGS="--steps 10 --scenario ObstacleAvoidance --agents 5 --envs 512" bash scripts/ab_bench.sh > gpurun_out/r06_wtrest_c5n5.log 2>&1 || exit 1
cp gpurun_out/ab.jsonl gpurun_out/r06_wtrest_c5n5.jsonl
python tools/ab_summary.py gpurun_out/r06_wtrest_c2.jsonl gpurun_out/r06_wtrest_c3.jsonl gpurun_out/r06_wtrest_c5.jsonl gpurun_out/r06_wtrest_c5n5.jsonl
