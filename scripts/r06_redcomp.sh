#!/bin/bash
# Round 6: the compensated (TwoSum) slab sum (SWARM_RED_COMP): the large parity tests and the
# fused / 3-launch / unfused equality tests against the variant library (margins recorded in
# gpurun_out/parity_errors.redcomp.json), then the interleaved A/B.
# NOTE: the SWARM_RED_COMP knob was removed after this A/B (f398917); its sources are at 97c9fb3, so rebuilding the variants from today's tree builds the product library.
export TMPDIR=/tmp
mkdir -p gpurun_out
SWARM_LIB_PATH=$PWD/ab/libswarm_redcomp.so SWARM_PARITY_ERRORS=gpurun_out/parity_errors.redcomp.json timeout -k 10 600 python -u -m pytest tests/test_gpu_parity_large.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "benchmark_size or one_launch or fused or unfused or td_" > gpurun_out/pytest_redcomp.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_redcomp.log; if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/pytest_redcomp.log | head -20; exit $rc; fi
TAG=redcomp V="base redcomp" V3="base redcomp" V5="base redcomp" REPS=3 bash scripts/r06_ab.sh || exit $?
python tools/ab_summary.py gpurun_out/r06_redcomp_c2.jsonl gpurun_out/r06_redcomp_c3.jsonl gpurun_out/r06_redcomp_c5.jsonl
