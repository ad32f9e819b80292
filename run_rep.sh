#!/bin/bash
export TMPDIR=/tmp
for i in 1 2 3; do
timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-timing > gpurun_out/bench_r.log 2>&1; rc=$?; tail -1 gpurun_out/bench_r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'])"
done
