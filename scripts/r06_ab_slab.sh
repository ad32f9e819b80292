#!/bin/bash
# Round 6: interleaved A/B of the slab-store modes (SWARM_SLAB_MODE, tools/ab_build.py variants)
# at C2, C3 and C5's N = 12 shard, then the instruction-fetch counters of base and preall, each
# counter set in its own rocprofv3 pass.  Stops at the first failure.
# NOTE: the SWARM_SLAB_MODE knob was removed after this A/B (642ba79); its sources are at b67f329, so rebuilding the variants from today's tree builds the product library.
export TMPDIR=/tmp
mkdir -p gpurun_out
V=${V:-"base slabsc1 slabplain4 slabnt4"}
VARIANTS="$V" REPS=${REPS:-3} BENCH_ARGS="--steps 20" bash scripts/ab_bench.sh > gpurun_out/r06_slab_c2.log 2>&1 || { tail -20 gpurun_out/r06_slab_c2.log; exit 1; }
cp gpurun_out/ab.jsonl gpurun_out/r06_slab_c2.jsonl
VARIANTS="$V" REPS=2 BENCH_ARGS="--steps 10 --scenario ObstacleAvoidance --agents 12" bash scripts/ab_bench.sh > gpurun_out/r06_slab_c3.log 2>&1 || { tail -20 gpurun_out/r06_slab_c3.log; exit 1; }
cp gpurun_out/ab.jsonl gpurun_out/r06_slab_c3.jsonl
VARIANTS="$V" REPS=2 BENCH_ARGS="--steps 10 --scenario ObstacleAvoidance --agents 12 --envs 512" bash scripts/ab_bench.sh > gpurun_out/r06_slab_c5.log 2>&1 || { tail -20 gpurun_out/r06_slab_c5.log; exit 1; }
cp gpurun_out/ab.jsonl gpurun_out/r06_slab_c5.jsonl
echo "slab ab ok"
if [ -n "$IFETCH" ]; then
for v in base preall; do
  if [ "$v" = base ]; then lib=""; else lib="$PWD/ab/libswarm_$v.so"; fi
  i=0
  for set in "InstrFetchLatency" "SQ_IFETCH SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY" "SQC_ICACHE_MISSES SQC_ICACHE_HITS"; do
    i=$((i+1))
    SWARM_LIB_PATH=$lib timeout -k 5 -s KILL 100 rocprofv3 --kernel-trace --pmc $set -d gpurun_out/r06_ifetch_$v/p$i -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-kernel-timing > gpurun_out/r06_ifetch_${v}_p$i.log 2>&1
    rc=$?; echo "ifetch $v pass $i rc=$rc"
    if [ $rc -ne 0 ]; then grep -v "^    @" gpurun_out/r06_ifetch_${v}_p$i.log | tail -4; exit $rc; fi
  done
done
fi
echo "done"
