// swarm_peer.h — the data-parallel tick's one exchange as peer stores over
// xGMI instead of an RCCL all_reduce launch: device side.  gfx950 only.
//
// Exchange buffer of one rank (uncached device memory, swarm_peer_alloc), 8-byte granules
// {hi: tag, lo: fp32 bits} (the fused tick's hand-off format, swarm_common.h):
//     [region 2][parity 2][source rank SWARM_PEER_MAX][kPeerCols]
// region 0 = swarm_reduce_advance_peer, region 1 = swarm_peer_allreduce; each region has its own
// launch counters (seq words [0, 128) and [128, 256)), so the two kinds never see each other's
// tags.  A column block with counter s publishes tag s + 1 into parity s & 1 of every rank's
// buffer, then polls its own.  Parity is enough: rank A can only publish launch s + 2 after every
// rank published launch s + 1, which each rank does only after its launch s (that read parity
// s & 1) has completed (stream order).
#pragma once

#include "swarm_common.h"

namespace swarm {

constexpr int kPeerCols = ((N_PARAMS + 1 + 15) / 16) * 16;   // 1680 columns per source rank
constexpr int kPeerSeqRegion = 128;                          // seq words per region
__host__ __device__ constexpr size_t peer_granules() { return (size_t)2 * 2 * SWARM_PEER_MAX * kPeerCols; }
constexpr uint32_t kPeerDefaultTimeoutUs = 5000000u;         // ranks enter the first tick skewed

__device__ inline unsigned long long* peer_slot(void* buf, int region, uint32_t parity, int src, int col) {
  return reinterpret_cast<unsigned long long*>(buf) +
         (((size_t)region * 2 + parity) * SWARM_PEER_MAX + src) * kPeerCols + col;
}

// one system-scope 8-byte store: the granule reaches the owner's memory whole (tag and value
// together), written through to the remote HBM over xGMI
__device__ inline void peer_put(void* buf, int region, uint32_t parity, int src, int col, uint32_t tag, float v) {
  const unsigned long long g = ((unsigned long long)tag << 32) | __float_as_uint(v);
  __hip_atomic_store(peer_slot(buf, region, parity, src, col), g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// poll this rank's own (uncached) buffer until the granule carries `tag`; bounded by the chip's
// 100 MHz clock, an expired wait counts in *err, sets *expired and yields 0
__device__ inline float peer_wait(void* own, int region, uint32_t parity, int src, int col, uint32_t tag,
                                  int32_t* err, uint32_t timeout_us, bool* expired) {
  const unsigned long long* g = peer_slot(own, region, parity, src, col);
  unsigned long long v = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if ((uint32_t)(v >> 32) != tag) {
    const uint64_t limit = (uint64_t)(timeout_us ? timeout_us : kPeerDefaultTimeoutUs) * 100u;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
      __builtin_amdgcn_s_sleep(2);
      v = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if ((uint32_t)(v >> 32) == tag) break;
      if (__builtin_amdgcn_s_memrealtime() - t0 > limit) {
        atomicAdd(err, 1);
        *expired = true;
        return 0.0f;
      }
    }
  }
  return __uint_as_float((uint32_t)v);
}

// The exchange of one column block: `mine` = this rank's value of column `col` (valid in the
// threads with q == 0 via the LDS row `mine_l`), threads q < W publish it to rank q and collect
// rank q's value; the caller then sums rv[0..W) in rank order.  blockDim = kCols * (>= W) threads
// indexed (q = tid / kCols, c = tid % kCols).  Ends with a block barrier.  hold != nullptr
// (swarm_reduce_advance_peer: &ctrl->peer_hold): an expired wait of the block sets it to 1.
template <int kCols>
__device__ inline void peer_exchange(const swarm_peer& P, int region, int blk, int q, int c, int col, int ncols,
                                     const float* mine_l, float (*rv)[kCols], uint32_t* hold = nullptr) {
  __shared__ int any_expired;
  const uint32_t s = P.seq[region * kPeerSeqRegion + blk];
  const uint32_t tag = s + 1u, parity = s & 1u;
  const int W = P.world_size;
  if (threadIdx.x == 0) any_expired = 0;
  __syncthreads();
  if (q < W && col < ncols) {
    bool expired = false;
    peer_put(P.recv[q], region, parity, P.rank, col, tag, mine_l[c]);
    rv[q][c] = peer_wait(P.recv[P.rank], region, parity, q, col, tag, P.err, P.timeout_us, &expired);
    if (expired) any_expired = 1;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    P.seq[region * kPeerSeqRegion + blk] = s + 1u;
    if (hold && any_expired) *hold = 1u;   // sticky; read by the next launch's optimizer step
  }
}

// host-side argument check of the peer entry points
inline int check_peer(const swarm_peer* p) {
  if (!p || p->world_size < 1 || p->world_size > SWARM_PEER_MAX || p->rank < 0 || p->rank >= p->world_size ||
      !p->seq || !p->err)
    return SWARM_E_BADARG;
  for (int q = 0; q < p->world_size; ++q)
    if (!p->recv[q]) return SWARM_E_BADARG;
  return 0;
}

}  // namespace swarm
