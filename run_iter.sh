#!/bin/bash
# one optimisation iteration on the GPU box: parity tests, stamps, bench + rocprof stats
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/pytest_gpu.log | head -20; exit $rc; fi
timeout -k 10 300 python tools/stamps.py > gpurun_out/stamps.log 2>&1; rc=$?; echo "stamps rc=$rc"
if [ $rc -ne 0 ]; then tail -5 gpurun_out/stamps.log; exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/iter -o run --output-format csv -- python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-kernel-timing > gpurun_out/iter_prof.log 2>&1
rc=$?; echo "prof rc=$rc"
if [ $rc -ne 0 ]; then tail -5 gpurun_out/iter_prof.log; exit $rc; fi
timeout -k 10 300 python bench.py --steps 400 --warmup 20 --no-cpu-baseline --no-kernel-timing > gpurun_out/iter_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -o '"value": [0-9.]*, "unit": "[a-z-/]*", "n_gpus": [0-9]*, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' gpurun_out/iter_bench.log
exit $rc
