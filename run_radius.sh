#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/pytest_gpu.log | head -30; exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_fused.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_fused.log | cut -c1-300
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/sweep.py gpurun_out/sweep_radius.jsonl radius > gpurun_out/sweep_radius.log 2>&1
rc=$?; cat gpurun_out/sweep_radius.log; exit $rc
