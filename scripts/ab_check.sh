#!/bin/bash
# A/B with a correctness gate: each non-base variant first runs the fused-tick parity subset
# (SWARM_LIB_PATH), then scripts/ab_bench.sh interleaves the bench runs.  VARIANTS="base x y".
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in $VARIANTS; do
  [ "$v" = base ] && continue
  SWARM_LIB_PATH=$PWD/ab/libswarm_$v.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
    -k "one_launch or fused or capture or td_ or two_rank or peer_tick or benchmark_size" > gpurun_out/ab_tests_$v.log 2>&1
  rc=$?; echo "variant $v tests rc=$rc"; tail -2 gpurun_out/ab_tests_$v.log
  if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/ab_tests_$v.log | head -20; exit $rc; fi
done
bash scripts/ab_bench.sh
