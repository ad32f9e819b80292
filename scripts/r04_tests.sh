#!/bin/bash
# round 4: the new and changed GPU parity tests first (verbose), then the tick split
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_parity_act_large.py tests/test_gpu_parity_large.py tests/test_compat_dropin.py \
  "tests/test_gpu_parity.py::test_closed_loop_rollout_reproduces_recorded_episodes" \
  "tests/test_gpu_parity.py::test_td_update_parity" "tests/test_gpu_parity.py::test_seed_set_after_construction_reaches_the_fused_tick" \
  > gpurun_out/pytest_new.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_new.log
cp gpurun_out/parity_errors.gpu.json gpurun_out/parity_errors_new.json 2>/dev/null
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/tick_split_stamps.py 1024 8 > gpurun_out/tick_split_rt.json 2> gpurun_out/tick_split_rt.err
rc=$?; echo "split rc=$rc"; head -16 gpurun_out/tick_split_rt.json; tail -3 gpurun_out/tick_split_rt.err
exit $rc
