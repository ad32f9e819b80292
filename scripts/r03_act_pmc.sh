#!/bin/bash
# kNN acting-rollout PMC passes (kernel-trace only beside --pmc), per library variant:
# VARIANTS="base notie" bash scripts/r03_act_pmc.sh  (base = the in-tree library, else ab/libswarm_<v>.so)
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/actpmc}
mkdir -p $OUT
ARGS="--mode act --graph knn --knn-k 5 --steps 5 --warmup 1 --no-cpu-baseline --no-kernel-timing"
for v in ${VARIANTS:-base}; do
  i=0
  for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_IFETCH SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY" \
             "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE" \
             "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS"; do
    i=$((i+1))
    if [ "$v" = base ]; then unset SWARM_LIB_PATH; else export SWARM_LIB_PATH=$PWD/ab/libswarm_$v.so; fi
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set -d $OUT/$v/p$i -o run --output-format csv -- python bench.py $ARGS > $OUT/$v.p$i.log 2>&1
    rc=$?; echo "$v pass $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $OUT/$v.p$i.log; exit $rc; fi
  done
done
python3 - <<'PY'
import csv, glob, collections, statistics, os
out = os.environ.get("OUT", "gpurun_out/actpmc")
vals = collections.defaultdict(list)
for f in glob.glob(f"{out}/*/p*/**/run_counter_collection.csv", recursive=True):
    v = f[len(out) + 1:].split("/")[0]
    for r in csv.DictReader(open(f)):
        if "act_kernel" in r["Kernel_Name"]:
            vals[(r["Counter_Name"], v)].append(float(r["Counter_Value"]))
for (c, v), x in sorted(vals.items()):
    print(f"{c:28s} {v:8s} {statistics.median(x):14.0f}  (n={len(x)})")
PY
