#!/bin/bash
# Round 5 interleaved A/B of source trees (tools/ab_trees.py): $VARIANTS (comma list of tree dirs),
# $ROUNDS rounds at C2 and, if $C3 is set, at C3 (OA 12 x 1024).  Stops at the first failure.
export TMPDIR=/tmp
mkdir -p gpurun_out
V=${VARIANTS:-abx/base,.}
timeout -k 10 1000 python -u tools/ab_trees.py gpurun_out/ab_c2.jsonl ${ROUNDS:-3} $V --steps 40 --no-cpu-baseline || exit $?
if [ -n "$C3" ]; then
timeout -k 10 1000 python -u tools/ab_trees.py gpurun_out/ab_c3.jsonl ${C3} $V --steps 20 --no-cpu-baseline --scenario ObstacleAvoidance --agents 12 || exit $?
fi
if [ -n "$C5" ]; then
timeout -k 10 1000 python -u tools/ab_trees.py gpurun_out/ab_c5.jsonl ${C5} $V --steps 20 --no-cpu-baseline --scenario ObstacleAvoidance --agents 12 --envs 512 || exit $?
fi
if [ -n "$C5N5" ]; then
timeout -k 10 1000 python -u tools/ab_trees.py gpurun_out/ab_c5n5.jsonl ${C5N5} $V --steps 20 --no-cpu-baseline --scenario ObstacleAvoidance --agents 5 --envs 512 || exit $?
fi
echo "ab ok"
