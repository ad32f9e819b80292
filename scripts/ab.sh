#!/bin/bash
# Quick A/B on the GPU box (bash scripts/ab.sh; TL=1 adds the fused-tick timeline): the fused-tick
# parity tests, then the headline bench line with the fused tick and with the 3-launch tick.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "one_launch or fused or capture or td_ or handoff or two_rank" > gpurun_out/pytest_fused.log 2>&1
rc=$?; echo "fused tests rc=$rc"; tail -3 gpurun_out/pytest_fused.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/pytest_fused.log | head -20; exit $rc; fi
for i in 1 2 3; do
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_fused.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_fused.log | cut -c1-420
if [ $rc -ne 0 ]; then exit $rc; fi
done
timeout -k 10 300 python bench.py --no-cpu-baseline --tick 3 --no-kernel-timing > gpurun_out/bench_3.log 2>&1
rc=$?; echo "bench3 rc=$rc"; tail -1 gpurun_out/bench_3.log | cut -c1-300
if [ $rc -ne 0 ]; then exit $rc; fi
if [ -n "$TL" ]; then timeout -k 10 200 python tools/tick_timeline.py > gpurun_out/tl.log 2>&1; rc=$?; tail -50 gpurun_out/tl.log; fi
exit $rc
