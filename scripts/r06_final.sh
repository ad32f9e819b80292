#!/bin/bash
# Round 6 verification of the in-tree libraries, one box (call A): GPU tests, smoke, the default
# bench line, its rocprofv3 --kernel-trace --stats profile and trace split, bench.py's own 2-rank
# launch (scripts/round.sh); then the realtime-stamps tick split and the PMC passes of the default
# bench command summarised with the build identity (scripts/r04_split.sh).  Stops at the first failure.
bash scripts/round.sh || exit $?
bash scripts/r04_split.sh || exit $?
echo "final A ok"
