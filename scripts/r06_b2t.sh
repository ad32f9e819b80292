#!/bin/bash
# Round 6: the transposed B2 tiles with 16-B slab stores (SWARM_B2_T=1 plain, =2 write-through sc1):
# bit-for-bit against the in-tree library at C2, C3 and C5 N = 5 (tools/bitcmp.py), then the
# interleaved A/B at C2 / C3 / C5 N = 12.  Stops at the first failure.
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/r06_bitcmp.jsonl
for v in b2t b2tsc1; do
  for cfg in "GoTo 8 1024 6" "ObstacleAvoidance 12 1024 4" "ObstacleAvoidance 5 512 4"; do
    timeout -k 10 300 python tools/bitcmp.py base ab/libswarm_$v.so $cfg >> gpurun_out/r06_bitcmp.jsonl 2> gpurun_out/r06_bitcmp.err || { tail -5 gpurun_out/r06_bitcmp.err; exit 1; }
  done
done
cat gpurun_out/r06_bitcmp.jsonl | cut -c1-400
TAG=b2t V="base b2t b2tsc1" V3="base b2t b2tsc1" V5="base b2t b2tsc1" bash scripts/r06_ab.sh || exit $?
