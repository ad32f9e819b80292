"""Philox4x32-10 counter-based RNG, numpy restatement (TEST INFRASTRUCTURE ONLY).

The reference draws its exploration coins and random actions from Python's
``random`` module (``src/training/train_gcn_dqn.py:164-165``) and its reset
centres from the torch global RNG (``src/scenarios/go_to_position_scenario.py:88``).
Neither stream can be reproduced on a GPU, so the build keys every draw by
(seed, tick, env, stream) through Philox4x32-10 (Salmon et al., SC'11,
"Parallel random numbers: as easy as 1, 2, 3").  The HIP kernels
(``csrc/swarm_rng.h``) and this module implement the same integer function, so
the oracle reproduces the GPU's draws bit for bit.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s CPU baseline may
import anything under ``oracle/``.
"""
from __future__ import annotations

import numpy as np

PHILOX_M0 = np.uint64(0xD2511F53)
PHILOX_M1 = np.uint64(0xCD9E8D57)
PHILOX_W0 = np.uint32(0x9E3779B9)
PHILOX_W1 = np.uint32(0xBB67AE85)
MASK32 = np.uint64(0xFFFFFFFF)

# stream ids (third counter word); must match csrc/swarm_rng.h
STREAM_COIN = 1
STREAM_RAND_ACTION = 2
STREAM_RESET = 3
STREAM_SAMPLE = 4


def philox4x32(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10. All inputs broadcastable uint32 arrays/ints.

    Returns a tuple of four uint32 arrays.
    """
    c0 = np.asarray(c0, dtype=np.uint32).astype(np.uint64)
    c1 = np.asarray(c1, dtype=np.uint32).astype(np.uint64)
    c2 = np.asarray(c2, dtype=np.uint32).astype(np.uint64)
    c3 = np.asarray(c3, dtype=np.uint32).astype(np.uint64)
    k0 = np.asarray(k0, dtype=np.uint32).astype(np.uint64)
    k1 = np.asarray(k1, dtype=np.uint32).astype(np.uint64)
    c0, c1, c2, c3, k0, k1 = np.broadcast_arrays(c0, c1, c2, c3, k0, k1)
    c0, c1, c2, c3 = c0.copy(), c1.copy(), c2.copy(), c3.copy()
    k0, k1 = k0.copy(), k1.copy()
    for r in range(10):
        if r > 0:
            k0 = (k0 + np.uint64(PHILOX_W0)) & MASK32
            k1 = (k1 + np.uint64(PHILOX_W1)) & MASK32
        p0 = PHILOX_M0 * c0
        p1 = PHILOX_M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK32
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK32
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0) & MASK32, lo1, (hi0 ^ c3 ^ k1) & MASK32, lo0
    return (c0.astype(np.uint32), c1.astype(np.uint32),
            c2.astype(np.uint32), c3.astype(np.uint32))


def seed_key(seed: int):
    """Split a 64-bit seed into the two Philox key words (csrc: swarm_key)."""
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    return np.uint32(seed & 0xFFFFFFFF), np.uint32(seed >> 32)


def u01(word):
    """uint32 -> float32 uniform in [0, 1): top 24 bits times 2^-24 (exact)."""
    w = np.asarray(word, dtype=np.uint32)
    return ((w >> np.uint32(8)).astype(np.float32) * np.float32(2.0 ** -24)).astype(np.float32)


def uniform_int(word, n: int):
    """uint32 -> integer in [0, n): (word * n) >> 32 (csrc: swarm_uniform_int)."""
    w = np.asarray(word, dtype=np.uint32).astype(np.uint64)
    return ((w * np.uint64(n)) >> np.uint64(32)).astype(np.int64)
