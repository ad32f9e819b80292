#!/bin/bash
# One verification pass on the GPU box: gpu parity tests, smoke, the default bench line, the
# rocprofv3 --kernel-trace --stats profile of the same bench command (csv, so that
# tools/trace_split.py can split the tick by dispatch start stamps), and bench.py's own
# multi-rank launch (two gloo ranks sharing the one GPU, started by bench.py itself).
# Stops at the first failure.
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/pytest_gpu.log | head -20; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
fi
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_default.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/final_prof -o run --output-format csv -- python bench.py --no-cpu-baseline > gpurun_out/final_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -1 gpurun_out/final_prof.log
if [ $rc -ne 0 ]; then exit $rc; fi
python tools/trace_split.py gpurun_out/final_prof/run_kernel_trace.csv gpurun_out/trace_split.json > gpurun_out/trace_split.log 2>&1
echo "trace_split rc=$?"; cat gpurun_out/trace_split.log | head -40
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --steps 2 --no-cpu-baseline --no-kernel-timing > gpurun_out/bench_spawn2.log 2>&1
rc=$?; echo "bench --gpus 2 (self-spawned gloo ranks) rc=$rc"; tail -1 gpurun_out/bench_spawn2.log
exit $rc
