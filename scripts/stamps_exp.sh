export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/stamps.py > gpurun_out/stamps_1024.log 2>&1 || exit 1
ENVS=64 timeout -k 10 200 python tools/stamps.py > gpurun_out/stamps_64.log 2>&1 || exit 1
timeout -k 10 200 python tools/tick_timeline.py 1024 > gpurun_out/timeline_1024.log 2>&1 || exit 1
echo ok
