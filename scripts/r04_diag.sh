#!/bin/bash
# round 4 diagnostics: realtime-stamps tick split and segment-stamps timelines at C2 and the C5
# shard (OA 5 / 12 agents x 512 envs), current tree's diagnostic builds
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "1024 8 GoTo gat" "512 12 ObstacleAvoidance gat" "512 5 ObstacleAvoidance gat" "512 12 ObstacleAvoidance gcn"; do
  tag=$(echo $cfg | tr ' ' '_')
  timeout -k 10 300 python tools/tick_split_stamps.py $cfg > gpurun_out/split_$tag.json 2> gpurun_out/split_$tag.err
  rc=$?; echo "split $tag rc=$rc"; python -c "import json; print(json.load(open('gpurun_out/split_$tag.json'))['median_of_5'])"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/split_$tag.err; exit $rc; fi
done
for cfg in "1024 8 GoTo gat" "512 12 ObstacleAvoidance gat" "512 5 ObstacleAvoidance gat"; do
  tag=$(echo $cfg | tr ' ' '_')
  timeout -k 10 300 python tools/tick_timeline.py $cfg > gpurun_out/timeline_$tag.txt 2>&1
  rc=$?; echo "timeline $tag rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/timeline_$tag.txt; exit $rc; fi
done
