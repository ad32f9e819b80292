#!/bin/bash
# Round 6 diagnostic: the reduce launch's per-kind block ends (column, control, copy-back blocks)
# from a worktree build whose control and copy-back blocks also stamp their exit (abx/diag).
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/abx/diag/experiments-2025-acsos-marl-for-swarming-behaviors_amd/libswarm_hip_rtstamps.so
SWARM_SPLIT_LIB=$L timeout -k 10 300 python tools/tick_split_stamps.py 1024 8 > gpurun_out/r06_split_kinds_c2.json 2> gpurun_out/r06_split_kinds.err || exit 1
SWARM_SPLIT_LIB=$L timeout -k 10 300 python tools/tick_split_stamps.py 1024 12 ObstacleAvoidance > gpurun_out/r06_split_kinds_c3.json 2>> gpurun_out/r06_split_kinds.err || exit 1
python - <<'PY'
import json
for f in ("c2", "c3"):
    d = json.load(open("gpurun_out/r06_split_kinds_%s.json" % f))
    print(f, d["median_of_5"])
PY
