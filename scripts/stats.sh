#!/bin/bash
# Statistical parity of the training path and of the evaluation harness against the reference's
# recorded data (tools/train_parity.py, tools/eval_sweep.py).
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 800 python -u tools/train_parity.py --out gpurun_out/train_parity.json --agents 5,10 > gpurun_out/train_parity.log 2>&1
rc=$?; cat gpurun_out/train_parity.log | tail -12
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/eval_sweep.py /tmp/eval_sweep > gpurun_out/eval_sweep.log 2>&1
rc=$?; tail -22 gpurun_out/eval_sweep.log; cp /tmp/eval_sweep/summary.json gpurun_out/eval_sweep_summary.json; exit $rc
