// swarm_wpg.h — "wave per graph": one wave (64 lanes) owns ONE environment or
// sampled graph of up to NS node slots (NS = 8, 16, 32).  Lane l works on node slot
// s = l / G (G = 64 / NS lanes per slot) and owns the FPL = 32 / G contiguous hidden
// features [f0, f0 + FPL), f0 = FPL * (l % G).
//
// Per-node vectors are therefore 4 (NS = 8) to 16 (NS = 32) registers per lane and
// every dense per-node product is a k-ordered fmaf chain on the VALU; the full
// 32-vector of a slot that a product needs is exchanged through a per-wave LDS row.
// Reductions over a slot's feature groups are DPP butterflies (bitwise identical in
// every lane of the slot); graph-wide exchange (scores, positions, Q rows) goes
// through wave-private LDS with wave-scope syncs only — no workgroup barrier.
//
// GCN.forward: src/training/train_gcn_dqn.py:59-70 (GATConv -> tanh -> lin1 -> relu
// -> lin2); GATConv math: PyG 2.5.3 (heads 1, add_self_loops False).
#pragma once
#include "swarm_common.h"
#include "swarm_knn.h"

namespace swarm {

constexpr int kRow = 36;   // floats per LDS row of a 32-vector (32 + 4 pad, 16-B aligned)

template <int NS>
struct Wpg {
  static_assert(NS == 8 || NS == 16 || NS == 32, "node slots per wave");
  static constexpr int G = 64 / NS;          // lanes per node slot
  static constexpr int FPL = kHidden / G;    // hidden features per lane
  static constexpr int F4 = FPL / 4;         // float4 per lane-slice
};

// Copy the flat parameter vector into an LDS image once per block (every weight
// read of the forward/backward then hits LDS).  All global loads are issued before
// the first LDS write and none sits behind a branch (clamped index): one round trip.
template <int NT>
struct ParamStage {
  // native 4-wide vectors: whole-float4 copies of HIP's float4 class lower to memcpys that
  // SROA leaves in scratch / promoted LDS once NJ > 1
  typedef float v4 __attribute__((ext_vector_type(4)));
  static constexpr int NF4 = N_PARAMS / 4;            // 418 full float4 (floats 0..1671)
  static constexpr int NJ = (NF4 + NT - 1) / NT;
  v4 v[NJ];
  float tail;
  __device__ inline void load(const float* __restrict__ g, int tid) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int i = min(tid + j * NT, NF4 - 1);
      v[j] = *reinterpret_cast<const v4*>(g + 4 * i);
    }
    tail = g[N_PARAMS - 1];
  }
  // into the padded LDS image (lds_index: lin1 / lin2 rows at a 36-float stride)
  __device__ inline void store(float* __restrict__ lds, int tid) const {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int i = tid + j * NT;
      if (i < NF4) *reinterpret_cast<v4*>(lds + lds_index(4 * i)) = v[j];
    }
    if (tid == 0) lds[lds_index(N_PARAMS - 1)] = tail;
  }
};
static_assert(ParamStage<64>::NF4 * 4 + 1 == N_PARAMS && N_PARAMS_PAD == ParamStage<64>::NF4 * 4 + 4, "tail");

// LDS traffic between lanes of ONE wave: LDS executes a wave's instructions in
// order, so only compiler reordering has to be fenced (rocPRIM's wave_barrier).
__device__ inline void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int CTRL>
__device__ inline float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}

// sum over the G contiguous lanes of a slot: quad_perm xor-1, xor-2, then
// row_half_mirror (lane i <-> 7 - i inside 8 lanes); a + b == b + a, so every lane
// of the slot ends with the bitwise same value.
template <int G>
__device__ inline float slot_sum(float x) {
  x = x + dppf<0xB1>(x);
  if constexpr (G >= 4) x = x + dppf<0x4E>(x);
  if constexpr (G >= 8) x = x + dppf<0x141>(x);
  static_assert(G == 2 || G == 4 || G == 8, "slot width");
  return x;
}

template <int NS>
struct WGeom {
  int lane, s, q, f0;
  int gid;      // env (acting) or batch index (TD) of this wave; 0 if the wave is idle
  bool live;    // the wave has a graph
  bool valid;   // live && s < N: this lane's slot is a real node
};

template <int NS>
__device__ inline WGeom<NS> make_wgeom(int wave_gid, int count, int N) {
  WGeom<NS> g;
  g.lane = threadIdx.x & 63;
  g.s = g.lane / Wpg<NS>::G;
  g.q = g.lane % Wpg<NS>::G;
  g.f0 = g.q * Wpg<NS>::FPL;
  g.live = wave_gid < count;
  g.gid = g.live ? wave_gid : 0;
  g.valid = g.live && g.s < N;
  return g;
}

// per-wave small LDS scratch
template <int NS>
struct WSmall {
  float Q[NS][12];
  float ssrc[NS], sdst[NS], px[NS], py[NS], aux[NS], aux2[NS];
  uint32_t knn[NS];
};

// an acting wave's kNN tie memo (knn_masks_wave): per slot, the rank signature of the last
// tie row it resolved and that row's neighbour set; sig_lo = ~0 marks an empty entry (no row
// has every rank 15)
template <int NS>
struct TieMemo {
  uint32_t sig_lo[NS], sig_hi[NS], mask[NS];
  __device__ void clear(int lane) {
    for (int n = lane; n < NS; n += 64) sig_lo[n] = ~0u;
  }
};

// what one wave's forward reads and writes in LDS: NS rows of H, T (tanh out) and
// R (relu out) — private scratch when acting, rows of the TD block's images in TD
template <int NS>
struct WView {
  float (*H)[kRow];
  float (*T)[kRow];
  float (*R)[kRow];
  WSmall<NS>* sm;
  TieMemo<NS>* memo = nullptr;   // acting waves only
};

template <int NS>
struct WScratch {
  float H[NS][kRow], T[NS][kRow], R[NS][kRow];
  WSmall<NS> sm;
  TieMemo<NS> memo;
  __device__ WView<NS> view() { return WView<NS>{H, T, R, &sm, &memo}; }
};

template <int K>
__device__ inline void lds_load(const float* __restrict__ p, float* out) {   // K floats, 16-B aligned
#pragma unroll
  for (int i = 0; i < K / 4; ++i) {
    const float4 v = reinterpret_cast<const float4*>(p)[i];
    out[4 * i] = v.x; out[4 * i + 1] = v.y; out[4 * i + 2] = v.z; out[4 * i + 3] = v.w;
  }
}
template <int K>
__device__ inline void lds_store(float* __restrict__ p, const float* in) {
#pragma unroll
  for (int i = 0; i < K / 4; ++i)
    reinterpret_cast<float4*>(p)[i] = make_float4(in[4 * i], in[4 * i + 1], in[4 * i + 2], in[4 * i + 3]);
}

// ---- MFMA 16x16x4 f32 ("D layout").  D = A B with A [16 rows][4 k], B [4 k][16 cols]:
// lane l supplies A[l & 15][kslot = l >> 4] and B[kslot = l >> 4][l & 15] and holds
// D[4 (l >> 4) + r][l & 15], r = 0..3.  Here the columns are the graph's node slots
// (column tile ct covers slots 16 ct .. 16 ct + 15) and the rows hidden features
// (row tile t covers 16 t .. 16 t + 15): lane l holds features 16 t + 4 p + r of node
// 16 ct + (l & 15), p = l >> 4.  A following product that sums over the feature index
// takes those registers as its B operand directly: k-step (t, r) pairs k-slot p with
// feature 16 t + 4 p + r.  Exact f32 (a k-ordered fmaf chain per instruction).
typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ inline f32x4 mfma16(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
template <int NS> struct Dl { static constexpr int CT = (NS + 15) / 16; };

// kNN row of slot s over the graph (simulator.py:17-19 -> CPU torch.topk set semantics)
template <int NS>
__device__ inline uint32_t knn_mask(const WGeom<NS>& g, int N, int k, const WSmall<NS>& sm, KV* q) {
  float d[NS];
  const float xi = sm.px[g.s], yi = sm.py[g.s];
#pragma unroll
  for (int j = 0; j < NS; ++j) d[j] = (j < N) ? norm2(sm.px[j] - xi, sm.py[j] - yi) : 0.0f;
  return topk_smallest_mask<NS>(d, N, k, q);
}

// multiplicity m(u -> s) of every source slot u (target = this lane's slot)
//   complete (train_gcn_dqn.py:101-108): u != v pairs plus one (0, 0) edge
//   kNN (simulator.py:15-24): (i -> j) and (j -> i) for j in S_i, plus (0, 0)
//   radius: u -> s for u != s within the radius (symmetric), plus (0, 0)
//   dense: caller-supplied [B][N][N] uint8
template <int NS>
__device__ inline void in_edges(const WGeom<NS>& g, int N, int graph, const WSmall<NS>& sm,
                                const uint8_t* __restrict__ dense, int mult[NS]) {
  const int s = g.valid ? g.s : 0;
  const uint32_t ks = (graph == SWARM_GRAPH_KNN) ? sm.knn[s] : 0u;
#pragma unroll
  for (int u = 0; u < NS; ++u) {
    int m = 0;
    if (u < N && g.valid) {
      if (graph == SWARM_GRAPH_COMPLETE) {
        m = (u != s ? 1 : 0) + ((u == 0 && s == 0) ? 1 : 0);
      } else if (graph == SWARM_GRAPH_KNN) {
        m = (int)((sm.knn[u] >> s) & 1u) + (int)((ks >> u) & 1u) + ((u == 0 && s == 0) ? 1 : 0);
      } else if (graph == SWARM_GRAPH_RADIUS) {
        m = (int)((sm.knn[s] >> u) & 1u) + ((u == 0 && s == 0) ? 1 : 0);
      } else {
        m = (int)dense[((size_t)g.gid * N + u) * N + s];
      }
    }
    mult[u] = m;
  }
}

}  // namespace swarm
