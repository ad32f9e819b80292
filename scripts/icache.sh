#!/bin/bash
# instruction-cache PMC passes over the bench workload (kernel-trace only beside --pmc)
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/icache}
mkdir -p $OUT
ARGS="--steps 5 --warmup 1 --no-cpu-baseline --no-kernel-timing"
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAIT_ANY" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set -d $OUT/p$i -o run --output-format csv -- python bench.py $ARGS > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done
python3 - <<'PY'
import csv,glob,collections,statistics
vals=collections.defaultdict(list)
for f in glob.glob('gpurun_out/icache/p*/run_counter_collection.csv'):
    for r in csv.DictReader(open(f)):
        k=r['Kernel_Name']
        key='tick' if 'tick_kernel' in k else 'act' if 'act_kernel' in k else 'td' if 'td_kernel' in k else 'red' if 'reduce' in k else None
        if key: vals[(key,r['Counter_Name'])].append(float(r['Counter_Value']))
for (k,c),v in sorted(vals.items()): print(k,c,statistics.median(v))
PY
