#!/bin/bash
# A/B helper: build the product library of an earlier commit into ab/libswarm_NAME.so
# usage: scripts/build_at.sh COMMIT NAME   (worktree under build/, removed afterwards)
set -e
c=$1; n=$2; root=$(git rev-parse --show-toplevel); wt=$root/build/wt_$n
rm -rf "$wt"; git worktree prune
git worktree add -f --detach "$wt" "$c" > /dev/null
pkg=experiments-2025-acsos-marl-for-swarming-behaviors_amd
(cd "$wt" && python -c "import sys; sys.path.insert(0, '$pkg'); sys.path.insert(0, '.'); import importlib.util as u; s=u.spec_from_file_location('b', '$pkg/build.py'); m=u.module_from_spec(s); s.loader.exec_module(m); m.build(force=True, verbose=False)")
mkdir -p "$root/ab"; cp "$wt/$pkg/libswarm_hip.so" "$root/ab/libswarm_$n.so"
git worktree remove --force "$wt"
echo "built ab/libswarm_$n.so from $(git rev-parse --short $c)"
