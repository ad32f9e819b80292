#!/bin/bash
# quick A/B: fused vs 3-launch bench lines (+ optional timeline)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_fused.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_fused.log | cut -c1-420
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline --tick 3 --no-kernel-timing > gpurun_out/bench_3.log 2>&1
rc=$?; echo "bench3 rc=$rc"; tail -1 gpurun_out/bench_3.log | cut -c1-300
if [ $rc -ne 0 ]; then exit $rc; fi
if [ -n "$TL" ]; then timeout -k 10 200 python tools/tick_timeline.py > gpurun_out/tl.log 2>&1; rc=$?; head -14 gpurun_out/tl.log; fi
exit $rc
