#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 40 --warmup 3 --no-cpu-baseline > gpurun_out/bench_head.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_head.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 1000 python -u tools/sweep.py gpurun_out/sweep.jsonl > gpurun_out/sweep.log 2>&1
rc=$?; cat gpurun_out/sweep.log | tail -25; exit $rc
