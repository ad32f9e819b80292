#!/bin/bash
# one-launch tick (SWARM_F_TICK_REDUCE): parity tests, then the headline bench with the reduce
# in-kernel (SWARM_TICK_REDUCE=1) against the two-launch tick (=0), interleaved
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread \
  -k "single_launch or one_launch_tick or handoff or large or trainer or two_rank or flush" > gpurun_out/red_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/red_tests.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/red_tests.log | head -30; exit $rc; fi
: > gpurun_out/ab_red.jsonl
for rep in $(seq ${REPS:-3}); do
  for v in 1 0; do
    SWARM_TICK_REDUCE=$v timeout -k 10 300 python bench.py --no-cpu-baseline $BENCH_ARGS > gpurun_out/ab_red_$v.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "variant $v rc=$rc"; tail -5 gpurun_out/ab_red_$v.log; exit $rc; fi
    python -c "import json; d=json.loads(open('gpurun_out/ab_red_$v.log').read().strip().splitlines()[-1]); print(json.dumps({'variant':'tick_reduce=$v','rep':$rep,'value':d['value'],'ms_per_step':d['ms_per_step'],'us_per_tick':d['us_per_tick'],'tick_us':d['tick_us'],'kernel_us':(d['roofline'] or {}).get('kernel_us'),'tick':d['config']['tick']}))" >> gpurun_out/ab_red.jsonl
  done
done
python -c "
import json
for l in open('gpurun_out/ab_red.jsonl'):
    d = json.loads(l); print(d['variant'], d['rep'], round(d['value'] / 1e6, 1), 'M', d['us_per_tick'], d['tick_us']['median'], d['kernel_us'])"
