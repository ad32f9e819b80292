#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "one_launch or fused or capture or td_" > gpurun_out/pytest_fused.log 2>&1
rc=$?; echo "fused tests rc=$rc"; tail -3 gpurun_out/pytest_fused.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/pytest_fused.log | head -20; exit $rc; fi
TL=$TL bash run_ab.sh
