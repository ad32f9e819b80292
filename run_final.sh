#!/bin/bash
# driver-equivalent round: smoke, the default bench line (cpu_baseline + roofline), and the
# rocprofv3 --kernel-trace --stats summary of the same bench command
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench_default.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/final_prof -o run --output-format csv -- python bench.py --no-cpu-baseline > gpurun_out/final_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
