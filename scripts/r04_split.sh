#!/bin/bash
# round 4: the un-profiled tick split from in-kernel realtime stamps, then the PMC passes of the
# default bench command for this build, summarised with the build identity
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/tick_split_stamps.py 1024 8 > gpurun_out/tick_split_stamps.json 2> gpurun_out/tick_split_stamps.err
rc=$?; echo "split rc=$rc"; cat gpurun_out/tick_split_stamps.json | head -20; tail -3 gpurun_out/tick_split_stamps.err
if [ $rc -ne 0 ]; then exit $rc; fi
OUT=gpurun_out/pmc bash scripts/pmc.sh
rc=$?; echo "pmc rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
python tools/pmc_summary.py gpurun_out/pmc gpurun_out/pmc_tick.json
