#!/bin/bash
# Round 5: instruction-cache counters of the fused tick (per dispatch), tree $TREE (default .)
export TMPDIR=/tmp
OUT=$(pwd)/gpurun_out/ic
mkdir -p $OUT
cd ${TREE:-.}
mkdir -p profiles
i=0
for set in "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_REQ SQC_TC_INST_REQ" "SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --pmc $set -d $OUT/p$i -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-kernel-timing > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done
