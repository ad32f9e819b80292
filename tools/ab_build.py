"""Build A/B variants of libswarm_hip.so into ab/ (git-ignored; travels to the GPU box):
python tools/ab_build.py name=-DFLAG=1,-DOTHER=2 [name2=...].  bench.py runs a variant with
SWARM_LIB_PATH=ab/libswarm_<name>.so (scripts/ab_bench.sh)."""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import swarm_amd  # noqa: E402,F401
from swarm_amd import build as b  # noqa: E402


def main():
    os.makedirs(os.path.join(ROOT, "ab"), exist_ok=True)
    jobs = []
    for arg in sys.argv[1:]:
        name, _, flags = arg.partition("=")
        jobs.append((os.path.join(ROOT, "ab", f"libswarm_{name}.so"), [f for f in flags.split(",") if f]))
    with ThreadPoolExecutor(max_workers=2) as ex:
        for out in ex.map(lambda j: b.build(force=True, verbose=False, out=j[0], extra=j[1]), jobs):
            print("built", out)


if __name__ == "__main__":
    main()
