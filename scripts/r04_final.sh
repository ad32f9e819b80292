#!/bin/bash
# round 4 final verification of the in-tree libraries: scripts/round.sh (GPU tests, smoke, default
# bench, rocprof stats + trace split, bench.py's own 2-rank launch), then scripts/r04_split.sh
# (realtime-stamps tick split, PMC passes summarised with the build identity), then stamps
# timelines at C2 and C3.  Stops at the first failure.
bash scripts/round.sh || exit $?
bash scripts/r04_split.sh || exit $?
timeout -k 10 300 python tools/tick_timeline.py 1024 8 GoTo gat > gpurun_out/timeline_final_1024_8.txt 2>&1 || exit $?
timeout -k 10 300 python tools/tick_timeline.py 1024 12 ObstacleAvoidance gat > gpurun_out/timeline_final_1024_12.txt 2>&1 || exit $?
echo "final ok"
