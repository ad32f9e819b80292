#!/bin/bash
# Rehearse bench.py's distributed path on a 1-GPU box: RCCL at one rank (graph-captured and eager
# all-reduce), and two gloo ranks sharing the GPU. Stops at the first failure.
export TMPDIR=/tmp
mkdir -p gpurun_out
R="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
A="--no-cpu-baseline --no-kernel-timing"
timeout -k 10 300 $R --nproc-per-node 1 --master-port 29511 bench.py --gpus 1 --force-dist $A > gpurun_out/dist_rccl1_graph.log 2>&1
rc=$?; echo "rccl1 graph rc=$rc"; tail -2 gpurun_out/dist_rccl1_graph.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 $R --nproc-per-node 1 --master-port 29512 bench.py --gpus 1 --force-dist --no-graph $A > gpurun_out/dist_rccl1_eager.log 2>&1
rc=$?; echo "rccl1 eager rc=$rc"; tail -1 gpurun_out/dist_rccl1_eager.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 $R --nproc-per-node 2 --master-port 29513 bench.py --gpus 2 --backend gloo --steps 2 --ticks 20 $A > gpurun_out/dist_gloo2.log 2>&1
rc=$?; echo "gloo2 rc=$rc"; tail -1 gpurun_out/dist_gloo2.log
exit $rc
