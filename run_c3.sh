#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/pytest_gpu.log | head -30; exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_fused.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_fused.log | cut -c1-200
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/sweep.py gpurun_out/sweep_c3.jsonl "C3 OA 12x1024 GAT train" > gpurun_out/sweep_c3.log 2>&1
rc=$?; cat gpurun_out/sweep_c3.log
timeout -k 10 300 python -u tools/sweep.py gpurun_out/sweep_c5.jsonl "C5 OA 12x512 GAT" > gpurun_out/sweep_c5.log 2>&1
rc=$?; cat gpurun_out/sweep_c5.log; exit $rc
