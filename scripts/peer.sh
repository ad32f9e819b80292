#!/bin/bash
# Peer all-reduce on the 1-GPU box: its GPU tests (in-process W-rank emulation, two-process HIP
# IPC), then bench.py's distributed path with it: one nccl rank (W = 1 exchange, graph-captured),
# two gloo ranks sharing the GPU (W = 2 exchange through IPC, graph-captured), and the same two
# ranks with the plain gloo all-reduce for comparison.  Stops at the first failure.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_peer.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/peer_tests.log 2>&1
rc=$?; echo "peer tests rc=$rc"; tail -16 gpurun_out/peer_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
R="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
A="--no-cpu-baseline --no-kernel-timing"
timeout -k 10 300 $R --nproc-per-node 1 --master-port 29521 bench.py --gpus 1 --force-dist --allreduce peer $A > gpurun_out/dist_peer1.log 2>&1
rc=$?; echo "peer W=1 rc=$rc"; tail -1 gpurun_out/dist_peer1.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 $R --nproc-per-node 2 --master-port 29522 bench.py --gpus 2 --backend gloo --allreduce peer --steps 5 $A > gpurun_out/dist_peer_gloo2.log 2>&1
rc=$?; echo "peer W=2 (2 processes, 1 GPU) rc=$rc"; tail -1 gpurun_out/dist_peer_gloo2.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 $R --nproc-per-node 2 --master-port 29523 bench.py --gpus 2 --backend gloo --allreduce rccl --steps 2 $A > gpurun_out/dist_gloo2.log 2>&1
rc=$?; echo "gloo all-reduce W=2 rc=$rc"; tail -1 gpurun_out/dist_gloo2.log
exit $rc
