export TMPDIR=/tmp
timeout -k 10 300 python tools/stamps.py > gpurun_out/stamps.log 2>&1; rc=$?; cat gpurun_out/stamps.log; exit $rc
