#!/bin/bash
export TMPDIR=/tmp
for cfg in "SWARM_TD_TPB=1" "SWARM_TD_TPB=2" "SWARM_TD_TPB=3" "SWARM_TD_TPB=2 SWARM_NO_GN=1"; do
  tag=$(echo $cfg | tr ' =' '__')
  env $cfg timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ab2_$tag -o run --output-format csv -- python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-kernel-timing > gpurun_out/ab2_$tag.log 2>&1
  rc=$?; echo "$cfg rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/ab2_$tag.log)"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
