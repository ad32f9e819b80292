#!/bin/bash
# Round 6 diagnostics (timing-only library variants from tools/ab_build.py, never shipped):
#  1. interleaved A/B at C2 (and C3): base vs fewslabs8 (only 8 TD blocks store slabs and the reduce
#     reads 8: the timing bound of any slab cut, VERDICT r5 "next" #3) vs preall (every TD block on
#     the hand-off blocks' pre path: the instruction-cache test of VERDICT r5 "next" #4);
#  2. the stamps timelines of base and preall (hand-off blocks' post-y stretch);
#  3. instruction-fetch counters of base and preall (InstrFetchLatency = accumulated SQ_IFETCH_LEVEL
#     / SQ_IFETCH, i.e. mean cycles per instruction fetch, and the L1I hit / miss counts).
# Stops at the first failure.
export TMPDIR=/tmp
mkdir -p gpurun_out
VARIANTS="base fewslabs8 preall" REPS=3 BENCH_ARGS="--steps 20" bash scripts/ab_bench.sh > gpurun_out/r06_ab_c2.log 2>&1 || { tail -20 gpurun_out/r06_ab_c2.log; exit 1; }
cp gpurun_out/ab.jsonl gpurun_out/r06_ab_c2.jsonl
VARIANTS="base fewslabs8" REPS=2 BENCH_ARGS="--steps 10 --scenario ObstacleAvoidance --agents 12" bash scripts/ab_bench.sh > gpurun_out/r06_ab_c3.log 2>&1 || { tail -20 gpurun_out/r06_ab_c3.log; exit 1; }
cp gpurun_out/ab.jsonl gpurun_out/r06_ab_c3.jsonl
echo "ab ok"; cat gpurun_out/r06_ab_c2.jsonl gpurun_out/r06_ab_c3.jsonl | cut -c1-200
timeout -k 10 200 python tools/tick_timeline.py > gpurun_out/r06_tl_base.txt 2>&1 || { tail -20 gpurun_out/r06_tl_base.txt; exit 1; }
SWARM_TL_LIB=$PWD/ab/libswarm_stamps_preall.so timeout -k 10 200 python tools/tick_timeline.py > gpurun_out/r06_tl_preall.txt 2>&1 || { tail -20 gpurun_out/r06_tl_preall.txt; exit 1; }
echo "timelines ok"
for v in base preall; do
  if [ "$v" = base ]; then lib=""; else lib="$PWD/ab/libswarm_$v.so"; fi
  SWARM_LIB_PATH=$lib timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --pmc InstrFetchLatency SQ_IFETCH SQ_WAVE_CYCLES SQ_WAVES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQC_ICACHE_MISSES SQC_ICACHE_HITS -d gpurun_out/r06_ifetch_$v -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-kernel-timing > gpurun_out/r06_ifetch_$v.log 2>&1
  rc=$?; echo "ifetch $v rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/r06_ifetch_$v.log; exit $rc; fi
done
echo "diag ok"
