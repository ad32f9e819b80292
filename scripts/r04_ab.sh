#!/bin/bash
# round 4: GPU tests of the in-tree library (TESTS="..." selects; default the fused / TD parity set),
# then an interleaved A/B of the headline bench (and C3 with AB_C3=1) over VARIANTS ("base" = the
# in-tree library, NAME = ab/libswarm_NAME.so); CONFIGS="a;b" replaces the bench argument sets
# (';'-separated, "" = the default C2 line)
export TMPDIR=/tmp
mkdir -p gpurun_out
TESTS=${TESTS:-"tests/test_gpu_parity_act_large.py tests/test_gpu_parity_large.py tests/test_compat_dropin.py tests/test_gpu_parity.py::test_closed_loop_rollout_reproduces_recorded_episodes tests/test_gpu_parity.py::test_td_update_parity tests/test_gpu_parity.py::test_seed_set_after_construction_reaches_the_fused_tick tests/test_gpu_parity.py::test_fused_tick_equals_unfused tests/test_gpu_parity.py::test_one_launch_tick_equals_three_launch_tick"}
if [ "$TESTS" != none ]; then
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu $TESTS > gpurun_out/pytest_new.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error" gpurun_out/pytest_new.log | tail -5
cp gpurun_out/parity_errors.gpu.json gpurun_out/parity_errors_new.json 2>/dev/null
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|assert" gpurun_out/pytest_new.log | head -30; exit $rc; fi
fi
VARIANTS=${VARIANTS:-"base r4v1"}
: > gpurun_out/ab.jsonl
CONFIGS=${CONFIGS:-";${AB_C3:+--scenario ObstacleAvoidance --agents 12}"}
IFS=';' read -r -a CFGS <<< "$CONFIGS"
for args in "${CFGS[@]}"; do
[ -z "$args" ] && [ -n "$SEEN_DEFAULT" ] && continue
[ -z "$args" ] && SEEN_DEFAULT=1
for rep in $(seq 1 ${REPS:-3}); do
  for v in $VARIANTS; do
    if [ "$v" = base ]; then lib=""; else lib="$PWD/ab/libswarm_$v.so"; fi
    SWARM_LIB_PATH=$lib timeout -k 10 300 python bench.py --no-cpu-baseline $args > gpurun_out/ab_$v.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "variant $v rc=$rc"; tail -5 gpurun_out/ab_$v.log; exit $rc; fi
    python -c "import json,sys; d=json.loads(open('gpurun_out/ab_$v.log').read().strip().splitlines()[-1]); print(json.dumps({'variant':'$v','args':'$args','rep':$rep,'value':d['value'],'us_per_tick':d.get('us_per_tick'),'tick_us':d.get('tick_us'),'kernel_us':(d['roofline'] or {}).get('kernel_us')}))" >> gpurun_out/ab.jsonl
  done
done
done
cat gpurun_out/ab.jsonl
