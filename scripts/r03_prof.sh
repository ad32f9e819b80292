#!/bin/bash
# rocprofv3 kernel-trace stats of the default bench command, then the PMC passes (each its own
# run, kernel-trace only beside --pmc), summarised into gpurun_out/pmc_tick.json
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -1 gpurun_out/prof_bench.log | cut -c1-300
if [ $rc -ne 0 ]; then exit $rc; fi
OUT=gpurun_out/pmc bash scripts/pmc.sh || exit $?
python tools/pmc_summary.py gpurun_out/pmc gpurun_out/pmc_tick.json
