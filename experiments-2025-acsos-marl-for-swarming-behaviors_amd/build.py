"""Build libswarm_hip.so in-tree with hipcc for gfx950 (no JIT cache; the .so
travels with the repository snapshot to the GPU box)."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
SOURCES = ["swarm_act.hip", "swarm_td.hip"]
HEADERS = ["swarm_common.h", "swarm_knn.h", "swarm_tile.h"]
OUT = os.path.join(HERE, "libswarm_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared",
         "-Wall", "-Wno-unused-function"]


def _deps():
    files = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    files.append(os.path.join(os.path.dirname(HERE), "include", "swarm_hip.h"))
    return files


def up_to_date() -> bool:
    if not os.path.exists(OUT):
        return False
    t = os.path.getmtime(OUT)
    return all(os.path.getmtime(f) <= t for f in _deps())


def build(force: bool = False, verbose: bool = True) -> str:
    if not force and up_to_date():
        return OUT
    cmd = [HIPCC, *FLAGS, "-o", OUT + ".tmp", *[os.path.join(CSRC, s) for s in SOURCES]]
    if verbose:
        print("[build]", " ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
