"""How often the kNN build's boundary-tie path runs in acting-only rollouts (diagnostic library
built with -DSWARM_DIAG_TIE_COUNT=1; tools/ab_build.py tiecnt=-DSWARM_DIAG_TIE_COUNT=1):

    SWARM_LIB_PATH=ab/libswarm_tiecnt.so python tools/tie_count.py [envs] [agents] [k] [episodes]

Prints the kNN builds (waves x ticks), the builds with a tie row, the tie rows, and per episode
the share of waves that met a tie."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import swarm_amd
    from swarm_amd import _lib
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    k = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    eps_n = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    lib = _lib.load()
    fn = lib.swarm_dbg_tie_counts
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
    out = (ctypes.c_ulonglong * 3)()
    w = torch.tensor(np.load(os.path.join(ROOT, "tests", "golden", "weights.npz"))["weights_go_to"][0])
    eng = swarm_amd.SwarmEngine("GoTo", N, B, seed=0, params=w, graph="knn", knn_k=k, learn=False, eps=0.0)
    prev = [0, 0, 0]
    for i in range(eps_n):
        eng.reset()
        eng.rollout(100, tick0=100 * i, eps=0.0)
        torch.cuda.synchronize()
        assert fn(out) == 0
        cur = [int(x) for x in out]
        d = [c - p for c, p in zip(cur, prev)]
        prev = cur
        print(f"episode {i}: kNN builds {d[0]}, with a tie row {d[1]} ({d[1] / max(d[0], 1):.3%}), tie rows {d[2]}",
              flush=True)
    fe = lib.swarm_dbg_tie_env
    fe.argtypes = [ctypes.POINTER(ctypes.c_uint)]
    per = (ctypes.c_uint * 4096)()
    assert fe(per) == 0
    arr = np.array(per[:B], dtype=np.int64)
    print(f"tie builds per env over {eps_n} episodes: max {arr.max()}, p99 {np.percentile(arr, 99):.0f}, "
          f"mean {arr.mean():.2f}; per episode: max {arr.max() / eps_n:.1f}")


if __name__ == "__main__":
    main()
