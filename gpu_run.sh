#!/bin/bash
# GPU-box driver for one measurement round: parity tests, smoke, bench. Stops after any crash.
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
else rc=0; fi
echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
if [ -n "$SKIP_BENCH" ]; then exit 0; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 200 --warmup 10 --cpu-seconds ${CPU_SECONDS:-10} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
exit $rc
