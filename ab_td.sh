#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
for w in 1 2 4; do
  SWARM_TD_WPB=$w timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab_w$w -o run --output-format csv -- python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-kernel-timing > gpurun_out/ab_w$w.log 2>&1
  rc=$?; echo "w=$w rc=$rc"; grep -o '"value": [0-9.]*' gpurun_out/ab_w$w.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
