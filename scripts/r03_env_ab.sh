#!/bin/bash
# launch-path environment A/B on the headline bench (per-tick time and the empty-kernel chain)
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/env_ab.txt
for rep in 1 2; do
  for e in "" "HIP_FORCE_DEV_KERNARG=1" "HIP_FORCE_DEV_KERNARG=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" "HIP_LAUNCH_BLOCKING=0 AMD_DIRECT_DISPATCH=1"; do
    env $e timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/env_ab.log 2>&1 || { tail -3 gpurun_out/env_ab.log; exit 1; }
    python - "$e" >> gpurun_out/env_ab.txt <<'PY'
import json, sys
d = json.loads(open("gpurun_out/env_ab.log").read().strip().splitlines()[-1])
kt = d["roofline"]["kernel_us"]
print(f"{sys.argv[1] or 'default':45s} tick {d['us_per_tick']:.3f} us  median {d['tick_us']['median']:.3f}  tick_kernel {kt['tick_kernel']:.2f}  advance {kt['ctrl_advance_kernel']:.2f}")
PY
  done
done
cat gpurun_out/env_ab.txt
