#!/bin/bash
# Round 6: the write-through B2-tile slab stores, hazard-padded asm (b2tsc1) and compiler-generated
# 8-B agent-scope stores (b2tx2): bit-for-bit against the in-tree library at C2, C3, C5 N = 5 and
# 12 (tools/bitcmp.py), then the interleaved A/B.  Stops at the first failure or mismatch.
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/r06_bitcmp2.jsonl
for v in b2tsc1 b2tx2 b2thyb; do
  for cfg in "GoTo 8 1024 6" "ObstacleAvoidance 12 1024 4" "ObstacleAvoidance 5 512 4" "ObstacleAvoidance 12 512 4" "GoTo 8 64 8"; do
    timeout -k 10 300 python tools/bitcmp.py base ab/libswarm_$v.so $cfg >> gpurun_out/r06_bitcmp2.jsonl 2> gpurun_out/r06_bitcmp2.err || { tail -5 gpurun_out/r06_bitcmp2.err; exit 1; }
  done
done
python -c "
import json
for l in open('gpurun_out/r06_bitcmp2.jsonl'):
    d = json.loads(l); print(d['b'], d['config'], d['all_bitwise'], d['grad_max_abs_diff'])
"
TAG=b2t2 V="base b2t b2tsc1 b2tx2 b2thyb" V3="base b2tsc1 b2tx2 b2thyb" V5="base b2tsc1 b2thyb" bash scripts/r06_ab.sh || exit $?
