"""Build libswarm_hip.so in-tree with hipcc for gfx950 (no JIT cache; the .so
travels with the repository snapshot to the GPU box)."""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
SOURCES = ["swarm_act.hip", "swarm_td.hip", "swarm_tick.hip", "swarm_peer.hip"]
HEADERS = ["swarm_actk.h", "swarm_tdk.h", "swarm_common.h", "swarm_knn.h", "swarm_wpg.h", "swarm_dl.h", "swarm_env.h",
           "swarm_adam.h", "swarm_gat3.h", "swarm_peer.h"]
OUT = os.path.join(HERE, "libswarm_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# kernarg preload: the leading 14 kernel-argument dwords arrive in SGPRs at wave start (the
# kernels put their first round trip's pointers there); older firmware runs the emitted
# compatibility prologue that loads them instead.
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared",
         "-Wall", "-Wno-unused-function", "-mllvm", "-amdgpu-kernarg-preload-count=14"]


def _deps():
    files = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    files += [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h") and f not in HEADERS]
    files.append(os.path.join(os.path.dirname(HERE), "include", "swarm_hip.h"))
    return files


def source_digest(extra=()) -> str:
    """sha256 (16 hex digits) of every source, header and compiler flag of a build: compiled into
    the library (swarm_build_info) so that a profile can name the code it measured."""
    h = hashlib.sha256()
    for f in sorted(_deps()):
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    h.update(" ".join(FLAGS + list(extra)).encode())
    return h.hexdigest()[:16]


def _current(out: str, extra=()) -> bool:
    """`out` is current: no source newer than it, or (a checkout touched the sources' times)
    it carries the digest of the sources and flags as they are now."""
    if not os.path.exists(out):
        return False
    t = os.path.getmtime(out)
    if all(os.path.getmtime(f) <= t for f in _deps()):
        return True
    with open(out, "rb") as f:
        return f"src {source_digest(extra)}".encode() in f.read()


def up_to_date() -> bool:
    return _current(OUT)


STAMPS_OUT = os.path.join(HERE, "libswarm_hip_stamps.so")
# test-only variant: every fused-tick hand-off wait overruns at once (tests of the drop path)
HODROP_OUT = os.path.join(HERE, "libswarm_hip_hodrop.so")
# test-only variant: the target waves' s' waits overrun at once, the online waves' r waits run to
# their bound (an overrun is counted once per dropping wave, not again by the r wait)
HODROP2_OUT = os.path.join(HERE, "libswarm_hip_hodrop2.so")
# test-only variant: 256-thread slab-reduce blocks (16 slab groups), so that eight ranks' peer
# reduces (each 109 blocks, all waiting on each other) are resident together on ONE GPU
# (tests/test_gpu_peer.py, the W = 8 fused exchange)
RED256_OUT = os.path.join(HERE, "libswarm_hip_red256.so")
# diagnostic variant: in-kernel realtime launch stamps only (tools/tick_split_stamps.py)
RTSTAMPS_OUT = os.path.join(HERE, "libswarm_hip_rtstamps.so")
VARIANTS = {"main": (OUT, []), "stamps": (STAMPS_OUT, ["-DSWARM_STAMPS=1"]),
            "rtstamps": (RTSTAMPS_OUT, ["-DSWARM_STAMPS=2"]), "hodrop": (HODROP_OUT, ["-DSWARM_HO_FORCE_DROP=1"]),
            "hodrop2": (HODROP2_OUT, ["-DSWARM_HO_FORCE_DROP=2"]), "red256": (RED256_OUT, ["-DSWARM_RED_GROUPS=16"])}
# the libraries the GPU tests load besides the main one (__graft_entry__.build builds them)
TEST_VARIANTS = ("hodrop", "hodrop2", "red256")


def build(force: bool = False, verbose: bool = True, stamps: bool = False, variant: str = "main",
          out: str = None, extra: list = None) -> str:
    """stamps=True (or variant="stamps") builds the diagnostic library (in-kernel s_memtime
    stamps); variant="hodrop" the hand-off overrun test library; out + extra: an A/B build
    (tools/ab_build.py) with extra compiler flags."""
    if out is None:
        out, extra = VARIANTS["stamps" if stamps else variant]
    extra = list(extra or [])
    if not force and _current(out, extra):
        return out
    # one hipcc process per translation unit (in parallel), then one link
    objs = [f"{out}.{os.path.splitext(src)[0]}.o" for src in SOURCES]
    cflags = [f for f in FLAGS if f != "-shared"] + [f'-DSWARM_SRC_DIGEST="{source_digest(extra)}"']
    procs = []
    for src, obj in zip(SOURCES, objs):
        cmd = [HIPCC, *cflags, *extra, "-c", "-o", obj, os.path.join(CSRC, src)]
        if verbose:
            print("[build]", " ".join(cmd), file=sys.stderr)
        procs.append(subprocess.Popen(cmd))
    if any(p.wait() != 0 for p in procs):
        raise subprocess.CalledProcessError(1, "hipcc")
    cmd = [HIPCC, "--offload-arch=gfx950", "-fPIC", "-shared", "-o", out + ".tmp", *objs]
    subprocess.run(cmd, check=True)
    for obj in objs:
        os.remove(obj)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    v = next((a[len("--variant="):] for a in sys.argv if a.startswith("--variant=")), "main")
    build(force="--force" in sys.argv, stamps="--stamps" in sys.argv, variant=v)
