#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 560 python -u tools/sweep.py gpurun_out/sweep.jsonl > gpurun_out/sweep.log 2>&1
rc=$?; cat gpurun_out/sweep.log | tail -25; exit $rc
