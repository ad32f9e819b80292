#!/bin/bash
# Round 5 diagnostics of the current build: realtime-stamps tick splits (C2, C3, C5 N=12 shard)
# and stamps timelines (C2, C3).  Stops at the first failure.
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "1024 8 GoTo gat" "1024 12 ObstacleAvoidance gat" "512 12 ObstacleAvoidance gat"; do
  tag=$(echo $cfg | tr ' ' '_')
  timeout -k 10 300 python tools/tick_split_stamps.py $cfg > gpurun_out/split_$tag.json 2> gpurun_out/split_$tag.err || { echo "split $tag failed"; tail -5 gpurun_out/split_$tag.err; exit 1; }
  echo "split $tag ok"
done
for cfg in "1024 8 GoTo gat" "1024 12 ObstacleAvoidance gat"; do
  tag=$(echo $cfg | tr ' ' '_')
  timeout -k 10 300 python tools/tick_timeline.py $cfg > gpurun_out/timeline_$tag.txt 2>&1 || { echo "timeline $tag failed"; tail -5 gpurun_out/timeline_$tag.txt; exit 1; }
  echo "timeline $tag ok"
done
