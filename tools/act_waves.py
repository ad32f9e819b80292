"""Diagnostic: per-wave lifetimes of the acting-only rollout and where each wave ran
(libswarm_hip_stamps.so: s_memrealtime at entry / exit, HW_ID + XCC_ID per wave).

    python tools/act_waves.py [envs] [agents] [graph] [k] [ticks]

Answers whether the launch's tail is a slow wave or waves sharing a SIMD / CU: prints the
lifetime distribution, the co-residency counts, and the lifetimes grouped by co-residency."""
import collections
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["SWARM_LIB_PATH"] = os.path.join(ROOT, "experiments-2025-acsos-marl-for-swarming-behaviors_amd",
                                            "libswarm_hip_stamps.so")
import numpy as np  # noqa: E402
import torch  # noqa: E402

import swarm_amd  # noqa: E402
from swarm_amd import _lib  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    graph = sys.argv[3] if len(sys.argv) > 3 else "knn"
    k = int(sys.argv[4]) if len(sys.argv) > 4 else 5
    ticks = int(sys.argv[5]) if len(sys.argv) > 5 else 100
    _lib.load()
    raw = ctypes.CDLL(_lib.LIB_PATH)
    raw.swarm_dbg_stamps_act.argtypes = [ctypes.c_void_p]
    w = torch.tensor(np.load(os.path.join(ROOT, "tests/golden/weights.npz"))["weights_go_to"][0])
    eng = swarm_amd.SwarmEngine("GoTo", N, B, seed=0, params=w, graph=graph, knn_k=k, learn=False, eps=0.0)
    sa = torch.zeros(4096 * 16 * 32, dtype=torch.int64, device="cuda")
    assert raw.swarm_dbg_stamps_act(sa.data_ptr()) == 0
    for rep in range(3):
        eng.reset()
        sa.zero_()
        eng.rollout(ticks, tick0=ticks * rep, eps=0.0)
        torch.cuda.synchronize()
        ab = (B + 3) // 4
        a = sa.cpu().numpy()[: ab * 16 * 32].reshape(ab, 16, 32)[:, :4].reshape(-1, 32)
        a = a[:B]
        st, en, hw = a[:, 30], a[:, 31], a[:, 29]
        life = (en - st) / 100.0
        span = (en.max() - st.min()) / 100.0
        hwid = hw & 0xFFFFFFFF
        xcc = (hw >> 32) & 0xF
        simd = (hwid >> 4) & 0x3
        cu = (hwid >> 8) & 0xF
        sh = (hwid >> 12) & 0x1
        se = (hwid >> 13) & 0x7
        cu_key = list(zip(xcc.tolist(), se.tolist(), sh.tolist(), cu.tolist()))
        simd_key = [c + (s,) for c, s in zip(cu_key, simd.tolist())]
        per_cu = collections.Counter(cu_key)
        per_simd = collections.Counter(simd_key)
        print(f"rollout {rep}: {B} waves, launch span {span:.1f} us; lifetime min {life.min():.1f} median "
              f"{np.median(life):.1f} p99 {np.percentile(life, 99):.1f} max {life.max():.1f} us; entry spread "
              f"{(st.max() - st.min()) / 100:.1f} us")
        print(f"  CUs used {len(per_cu)}, waves per CU {sorted(collections.Counter(per_cu.values()).items())}, "
              f"waves per SIMD {sorted(collections.Counter(per_simd.values()).items())}")
        share = np.array([per_simd[s] for s in simd_key])
        for c in sorted(set(share.tolist())):
            m = share == c
            print(f"  waves sharing their SIMD with {c - 1} other(s): {m.sum()} waves, lifetime median "
                  f"{np.median(life[m]):.1f} max {life[m].max():.1f} us")
        slow = np.argsort(-life)[:8]
        print("  slowest waves (env, lifetime us, waves on its SIMD, on its CU):",
              [(int(i), round(float(life[i]), 1), per_simd[simd_key[i]], per_cu[cu_key[i]]) for i in slow])
        # stamps-build counters (s_memtime cycles): tie-path entries, cycles in it, its slowest entry;
        # the wave's slowest tick and its index
        ties, tcyc, tmax, kmax, kidx, hits = a[:, 27], a[:, 28], a[:, 26], a[:, 25], a[:, 19], a[:, 18]
        print(f"  tie memo hits per wave (builds with at least one hit): mean {hits.mean():.2f} max {hits.max()}")
        print(f"  tie-path entries per wave: mean {ties.mean():.2f} max {ties.max()}; cycles per entry "
              f"{tcyc.sum() / max(ties.sum(), 1):.0f}; slowest entry {tmax.max()} cycles; slowest tick median "
              f"{np.median(kmax):.0f} max {kmax.max()} cycles")
        for i in slow[:6]:
            print(f"    env {int(i)}: {int(ties[i])} tie entries, {int(hits[i])} memo hits, {int(tcyc[i])} cycles in them (slowest {int(tmax[i])}); "
                  f"slowest tick {int(kidx[i])} at {int(kmax[i])} cycles")


if __name__ == "__main__":
    main()
