#!/bin/bash
# A/B: parity tests on the first library, then bench.py per library variant (ab/lib_*.so)
export TMPDIR=/tmp
mkdir -p gpurun_out
first=$1
SWARM_LIB_PATH=$PWD/ab/lib_$first.so timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/ab_pytest.log 2>&1
rc=$?; echo "pytest($first) rc=$rc"; tail -2 gpurun_out/ab_pytest.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/ab_pytest.log | head -20; exit $rc; fi
for rep in 1 2; do
for v in "$@"; do
  SWARM_LIB_PATH=$PWD/ab/lib_$v.so timeout -k 10 300 python bench.py --steps 400 --warmup 20 --no-cpu-baseline > gpurun_out/ab_$v.log 2>&1
  rc=$?; echo "$v rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/ab_$v.log) $(grep -o '"kernel_us": {[^}]*}' gpurun_out/ab_$v.log)"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/ab_$v.log; exit $rc; fi
done
done
