#!/bin/bash
# A/B of library variants (tools/ab_build.py -> ab/libswarm_<name>.so) on the headline bench:
# VARIANTS="base nt wt" bash scripts/ab_bench.sh; "base" = the in-tree library.  Each variant runs
# REPS times, interleaved, so drift hits all of them alike.  One JSON line per run.
export TMPDIR=/tmp
mkdir -p gpurun_out
REPS=${REPS:-3}
: > gpurun_out/ab.jsonl
for rep in $(seq $REPS); do
  for v in $VARIANTS; do
    if [ "$v" = base ]; then lib="$PWD/experiments-2025-acsos-marl-for-swarming-behaviors_amd/libswarm_hip.so"; else lib="$PWD/ab/libswarm_$v.so"; fi
    SWARM_LIB_PATH=$lib timeout -k 10 300 python bench.py --no-cpu-baseline $BENCH_ARGS > gpurun_out/ab_$v.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "variant $v rc=$rc"; tail -5 gpurun_out/ab_$v.log; exit $rc; fi
    python -c "import json,sys; d=json.loads(open('gpurun_out/ab_$v.log').read().strip().splitlines()[-1]); print(json.dumps({'variant':'$v','rep':$rep,'value':d['value'],'ms_per_step':d['ms_per_step'],'us_per_tick':d.get('us_per_tick'),'tick_us':d.get('tick_us'),'kernel_us':(d['roofline'] or {}).get('kernel_us')}))" >> gpurun_out/ab.jsonl
  done
done
cat gpurun_out/ab.jsonl
