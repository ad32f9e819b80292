#!/bin/bash
# round 3: the new parity / drop-in tests, then the training-parity agent sweep
export TMPDIR=/tmp
mkdir -p gpurun_out
SWARM_PARITY_ERRORS=gpurun_out/parity_errors_new.json timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_parity_large.py tests/test_compat_dropin.py "tests/test_gpu_parity.py::test_simulator_and_trainer_smoke" > gpurun_out/pytest_new.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_new.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python -u tools/train_parity.py --out gpurun_out/r03_train_parity_agents.json --scenarios ObstacleAvoidance,GoTo --agents ${AGENTS:-5,8,10,12} > gpurun_out/r03_train_parity_agents.txt 2>&1
rc=$?; echo "train_parity rc=$rc"; cat gpurun_out/r03_train_parity_agents.txt; exit $rc
