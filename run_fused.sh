#!/bin/bash
# fused-tick verification: its parity test first, then the whole GPU suite, then the bench
# line (fused) and the 3-launch A/B line.  Stops at the first failure.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "one_launch" > gpurun_out/pytest_fused.log 2>&1
rc=$?; echo "fused tests rc=$rc"; tail -12 gpurun_out/pytest_fused.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/pytest_gpu.log | head -20; exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_fused.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench_fused.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline --tick 3 > gpurun_out/bench_3.log 2>&1
rc=$?; echo "bench3 rc=$rc"; tail -1 gpurun_out/bench_3.log; exit $rc
