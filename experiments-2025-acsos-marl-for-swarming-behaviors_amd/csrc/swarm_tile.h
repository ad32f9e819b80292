// swarm_tile.h — one wave (64 lanes) owns a tile of 32 node slots = E = 32/N whole
// environments.  Lane l works on node slot v = l & 31; the two half-waves
// (h = l >> 5) hold complementary halves of every 32-wide hidden vector in the
// MFMA 32x32x2 f32 accumulator layout ("acc layout": register r of half h is
// hidden unit acc_row(r, h)).  Node-to-node traffic (neighbour H rows, scores,
// positions) goes through a per-wave LDS tile; the dense per-node MLP GEMMs
// (conv1.lin 7->32, lin1 32->32) run on MFMA; lin2 (32->9) and the attention
// softmax/aggregate run on the VALU with half-wave shuffle reductions.
//
// GCN.forward: src/training/train_gcn_dqn.py:59-70 (GATConv -> tanh -> lin1 ->
// relu -> lin2); GATConv math: PyG 2.5.3.
#pragma once
#include "swarm_common.h"
#include "swarm_knn.h"

namespace swarm {

constexpr int kHsStride = 36;   // floats per H row in LDS (32 + 4 pad, rows 16-B aligned)

struct WaveLds {
  float hs[kTile][kHsStride];   // H[node][hid], natural hidden order
  float ssrc[kTile];
  float sdst[kTile];
  float px[kTile], py[kTile];   // positions (graph build, collisions)
  float red[kTile];             // per-node scalar exchange (rewards, dis)
  float red2[kTile];
  uint32_t knn[kTile];          // kNN selection mask of each node slot
};

struct Geom {
  int lane, h, v;      // v = node slot
  int E;               // envs per tile
  int e_in_tile, agent, base;  // base = first slot of this lane's env
  int env;             // env index within the call (-1 if invalid)
  bool valid;
};

__device__ inline Geom make_geom(int tile, int N, int B) {
  Geom g;
  g.lane = threadIdx.x & 63;
  g.h = g.lane >> 5;
  g.v = g.lane & 31;
  g.E = kTile / N;
  g.e_in_tile = g.v / N;
  g.agent = g.v - g.e_in_tile * N;
  g.base = g.e_in_tile * N;
  const int env = tile * g.E + g.e_in_tile;
  g.valid = (g.e_in_tile < g.E) && (env < B);
  g.env = g.valid ? env : -1;
  if (!g.valid) { g.agent = 0; g.base = 0; }   // invalid lanes alias slot 0: in-bounds reads, no writes
  return g;
}

// ---------------------------------------------------------------- weights
// Copy the flat parameter vector into an LDS image once per block (every weight
// read of the forward/backward then hits LDS instead of a global round trip).
// All global loads are issued before the first LDS write and none sits behind a
// branch (clamped index), so the copy costs ONE memory round trip, not NJ.
template <int NT>
struct ParamStage {
  static constexpr int NF4 = N_PARAMS / 4;            // 418 full float4 (floats 0..1671)
  static constexpr int NJ = (NF4 + NT - 1) / NT;
  float4 v[NJ];
  float tail;
  __device__ inline void load(const float* __restrict__ g, int tid) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int i = min(tid + j * NT, NF4 - 1);
      v[j] = reinterpret_cast<const float4*>(g)[i];
    }
    tail = g[N_PARAMS - 1];
  }
  __device__ inline void store(float* __restrict__ lds, int tid) const {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int i = tid + j * NT;
      if (i < NF4) reinterpret_cast<float4*>(lds)[i] = v[j];
    }
    if (tid == 0) *reinterpret_cast<float4*>(lds + 4 * NF4) = make_float4(tail, 0.0f, 0.0f, 0.0f);
  }
};
static_assert(ParamStage<64>::NF4 * 4 + 1 == N_PARAMS && N_PARAMS_PAD == ParamStage<64>::NF4 * 4 + 4, "tail");

// float4 view of a 32-vector at the acc layout positions acc_row(4q..4q+3, h) = 8q+4h..+3
__device__ inline void load_vec_acc(const float* __restrict__ p, int h, float out[16]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4 w = *reinterpret_cast<const float4*>(p + 8 * q + 4 * h);
    out[4 * q + 0] = w.x; out[4 * q + 1] = w.y; out[4 * q + 2] = w.z; out[4 * q + 3] = w.w;
  }
}

// ---------------------------------------------------------------- graph
// multiplicity m(u -> v) for every source slot u of this lane's env (target v)
template <int NMAX>
__device__ inline void graph_mult(const Geom& g, int N, int graph, const WaveLds& L,
                                  const uint8_t* __restrict__ dense, int mult[NMAX]) {
#pragma unroll
  for (int u = 0; u < NMAX; ++u) {
    int m = 0;
    if (u < N && g.valid) {
      if (graph == SWARM_GRAPH_COMPLETE) {
        m = (u != g.agent ? 1 : 0) + ((u == 0 && g.agent == 0) ? 1 : 0);
      } else if (graph == SWARM_GRAPH_KNN) {
        const uint32_t su = L.knn[g.base + u];
        const uint32_t sv = L.knn[g.v];
        m = (int)((su >> g.agent) & 1u) + (int)((sv >> u) & 1u) + ((u == 0 && g.agent == 0) ? 1 : 0);
      } else {
        m = g.valid ? (int)dense[((size_t)g.env * N + u) * N + g.agent] : 0;
      }
    }
    mult[u] = m;
  }
}

// kNN row of this lane's node over its env (simulator.py:17-19); needs L.px/py
template <int NMAX>
__device__ inline uint32_t knn_row(const Geom& g, int N, int k, const WaveLds& L) {
  float d[NMAX];
  const float xi = L.px[g.v], yi = L.py[g.v];
#pragma unroll
  for (int j = 0; j < NMAX; ++j) {
    d[j] = 0.0f;
    if (j < N) d[j] = norm2(L.px[g.base + j] - xi, L.py[g.base + j] - yi);
  }
  return topk_smallest_mask<NMAX>(d, N, k);
}

// ---------------------------------------------------------------- forward
struct FwdState {
  float x[8];
  float hreg[16];
  float t[16];        // tanh(conv out)
  float zr[16];       // relu(lin1)
  float q[kActions];
  float sdst;
};

// H^T = W X^T on MFMA (K = 7 padded to 8): 4 x mfma_f32_32x32x2f32
__device__ inline void mfma_lin0(const float* __restrict__ P, const Geom& g, const float x[8], float hreg[16]) {
  f32x16 acc = {};
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int k = 2 * s + g.h;
    const float a = (k < kFeat) ? P[OFF_W + g.v * kFeat + k] : 0.0f;   // A[i = hid][k]
    const float b = g.h ? x[2 * s + 1] : x[2 * s];                      // B[k][j = node]
    acc = mfma32(a, b, acc);
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) hreg[r] = acc[r];
}

// Y^T = Wm X^T for a 32x32 weight (row-major [out][in]) and X^T in acc layout:
// K-step s pairs in-index acc_row(s,0) (half 0) with acc_row(s,1) (half 1).
__device__ inline void mfma_lin32(const float* __restrict__ Wm, const Geom& g, const float xin[16], float yout[16]) {
  float a[16];
  load_vec_acc(Wm + g.v * kHidden, g.h, a);       // A[i = out row l&31][k-slot] = Wm[i][acc_row(s,h)]
  f32x16 acc = {};
#pragma unroll
  for (int s = 0; s < 16; ++s) acc = mfma32(a[s], xin[s], acc);
#pragma unroll
  for (int r = 0; r < 16; ++r) yout[r] = acc[r];
}

// transpose-side product: Y^T = Wm^T X^T (Y[in] = sum_out Wm[out][in] X[out]), X in acc layout
__device__ inline void mfma_lin32_t(const float* __restrict__ Wm, const Geom& g, const float xin[16], float yout[16]) {
  f32x16 acc = {};
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const float a = Wm[acc_row(s, g.h) * kHidden + g.v];  // A[i = in col l&31][k-slot] = Wm[acc_row(s,h)][i]
    acc = mfma32(a, xin[s], acc);
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) yout[r] = acc[r];
}

// attention / aggregation for target node v. Writes c[u] = m_uv * alpha_uv (GAT) or the
// GCN normalisation (conv == GCN), and the aggregated conv output (before tanh) in out[16].
template <int NMAX>
__device__ inline void conv_aggregate(const float* __restrict__ P, const Geom& g, int N, int conv,
                                      WaveLds& L, const int mult[NMAX], float sdst, float c[NMAX],
                                      float out[16]) {
  if (conv == SWARM_CONV_GAT) {
    // branch-free over the env's sources u: every LDS read issued together, non-edges masked
    float e[NMAX];
    float emax = -INFINITY;
#pragma unroll
    for (int u = 0; u < NMAX; ++u) {
      const bool on = (u < N) && mult[u] > 0;
      e[u] = leaky(L.ssrc[g.base + (u < N ? u : 0)] + sdst);
      emax = on ? fmaxf(emax, e[u]) : emax;
    }
    float den = 0.0f;
#pragma unroll
    for (int u = 0; u < NMAX; ++u) {
      const bool on = (u < N) && mult[u] > 0;
      e[u] = on ? __expf(e[u] - emax) : 0.0f;
      den = den + (float)mult[u] * e[u];
    }
    den = den + 1e-16f;
    const float inv = 1.0f / den;
#pragma unroll
    for (int u = 0; u < NMAX; ++u) c[u] = (float)mult[u] * (e[u] * inv);
  } else {
    // GCNConv (a13, parity unpinned): self loops collapse to weight 1, deg on targets
    float deg = 0.0f;
#pragma unroll
    for (int u = 0; u < NMAX; ++u) {
      if (u < N) deg = deg + (u == g.agent ? 1.0f : (float)mult[u]);
    }
    const float dis = deg > 0.0f ? 1.0f / sqrtf(deg) : 0.0f;
    __syncthreads();
    if (g.h == 0) L.red2[g.v] = dis;
    __syncthreads();
#pragma unroll
    for (int u = 0; u < NMAX; ++u) {
      c[u] = 0.0f;
      if (u < N) {
        const float w = (u == g.agent ? 1.0f : (float)mult[u]);
        c[u] = (L.red2[g.base + u] * w) * dis;
      }
    }
  }
  float bias[16];
  load_vec_acc(P + OFF_BIAS, g.h, bias);
#pragma unroll
  for (int r = 0; r < 16; ++r) out[r] = 0.0f;
#pragma unroll
  for (int u = 0; u < NMAX; ++u) {
    if (u < N) {   // uniform condition; c[u] == 0 for non-edges
      const float* row = &L.hs[g.base + u][4 * g.h];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 hv = *reinterpret_cast<const float4*>(row + 8 * q);
        out[4 * q + 0] = out[4 * q + 0] + c[u] * hv.x;
        out[4 * q + 1] = out[4 * q + 1] + c[u] * hv.y;
        out[4 * q + 2] = out[4 * q + 2] + c[u] * hv.z;
        out[4 * q + 3] = out[4 * q + 3] + c[u] * hv.w;
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) out[r] = out[r] + bias[r];
}

// lin2 on MFMA: Q^T = W2 R^T with W2 zero-padded to 32 rows (A row a = l&31 < 9);
// result rows a = acc_row(r, h): half 0 holds a = 0..3 and 8, half 1 holds a = 4..7,
// exchanged with one xor-32 swap per value.
__device__ inline void lin2_mfma(const float* __restrict__ P, const Geom& g, const float zr[16], float q[kActions]) {
  float a[16];
  const int row = g.v < kActions ? g.v : 0;
  load_vec_acc(P + OFF_W2 + row * kHidden, g.h, a);
  if (g.v >= kActions) {
#pragma unroll
    for (int s = 0; s < 16; ++s) a[s] = 0.0f;
  }
  f32x16 acc = {};
#pragma unroll
  for (int s = 0; s < 16; ++s) acc = mfma32(a[s], zr[s], acc);
  // own: h0 -> {0,1,2,3,8} at r {0,1,2,3,4}; h1 -> {4,5,6,7} at r {0,1,2,3}
  const float o0 = acc[0], o1 = acc[1], o2 = acc[2], o3 = acc[3], o4 = acc[4];
  const float p0 = xor32(o0), p1 = xor32(o1), p2 = xor32(o2), p3 = xor32(o3), p4 = xor32(o4);
  float v[kActions];
  v[0] = g.h ? p0 : o0; v[1] = g.h ? p1 : o1; v[2] = g.h ? p2 : o2; v[3] = g.h ? p3 : o3;
  v[4] = g.h ? o0 : p0; v[5] = g.h ? o1 : p1; v[6] = g.h ? o2 : p2; v[7] = g.h ? o3 : p3;
  v[8] = g.h ? p4 : o4;
#pragma unroll
  for (int i = 0; i < kActions; ++i) q[i] = v[i] + P[OFF_B2 + i];
}

__device__ inline int argmax9(const float q[kActions]) {
  int best = 0;
  float bv = q[0];
#pragma unroll
  for (int a = 1; a < kActions; ++a)
    if (q[a] > bv) { bv = q[a]; best = a; }
  return best;
}

// Full GCN.forward for the tile.  Requires L.px/py written (kNN) for graph == KNN.
// Contains __syncthreads(): every lane of the block must call it.
template <int NMAX, int SB = -1>   // SB: diagnostic stamp base (SWARM_STAMPS builds only)
__device__ inline void tile_forward(const float* __restrict__ P, const Geom& g, int N, int graph, int k,
                                    int conv, const uint8_t* __restrict__ dense, WaveLds& L,
                                    FwdState& F, int mult[NMAX], float c[NMAX]) {
#define TF_STAMP(i) do { if (SB >= 0) SWARM_STAMP(SB + (i)); } while (0)
  mfma_lin0(P, g, F.x, F.hreg);
  float as[16], ad[16];
  load_vec_acc(P + OFF_ATT_SRC, g.h, as);
  load_vec_acc(P + OFF_ATT_DST, g.h, ad);
  float ps = 0.0f, pd = 0.0f;
#pragma unroll
  for (int r = 0; r < 16; ++r) { ps = ps + F.hreg[r] * as[r]; pd = pd + F.hreg[r] * ad[r]; }
  const float ssrc = ps + xor32(ps);
  F.sdst = pd + xor32(pd);
#pragma unroll
  for (int q = 0; q < 4; ++q)
    *reinterpret_cast<float4*>(&L.hs[g.v][8 * q + 4 * g.h]) =
        make_float4(F.hreg[4 * q], F.hreg[4 * q + 1], F.hreg[4 * q + 2], F.hreg[4 * q + 3]);
  if (g.h == 0) { L.ssrc[g.v] = ssrc; L.sdst[g.v] = F.sdst; }
  if (graph == SWARM_GRAPH_KNN) {
    const uint32_t m = g.valid ? knn_row<NMAX>(g, N, k, L) : 0u;
    if (g.h == 0) L.knn[g.v] = m;
  }
  TF_STAMP(0);
  __syncthreads();
  graph_mult<NMAX>(g, N, graph, L, dense, mult);
  TF_STAMP(1);
  float out[16];
  conv_aggregate<NMAX>(P, g, N, conv, L, mult, F.sdst, c, out);
  TF_STAMP(2);
#pragma unroll
  for (int r = 0; r < 16; ++r) F.t[r] = tanh_fast(out[r]);
  TF_STAMP(3);
  float z[16], b1[16];
  mfma_lin32(P + OFF_W1, g, F.t, z);
  load_vec_acc(P + OFF_B1, g.h, b1);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const float zz = z[r] + b1[r];
    F.zr[r] = zz > 0.0f ? zz : 0.0f;
  }
  TF_STAMP(4);
  lin2_mfma(P, g, F.zr, F.q);
  TF_STAMP(5);
#undef TF_STAMP
}

// ---------------------------------------------------------------- env step (one agent)
struct StepOut {
  float px, py, vx, vy;   // new state
  float dgoal;            // distance to goal after the step
  float dobs;             // World.get_distance(agent, obstacle) (OA)
};

// VMAS World.step for agent `agent` of an env whose pre-step positions are read
// through pos(u).  Force order: 0 + u, obstacle pair, agent pairs in ascending
// partner index; -f(p_u - p_v) == f(p_v - p_u) bit for bit.
template <int NMAX, typename PosFn>
__device__ inline StepOut agent_step(int scenario, int N, int agent, float px, float py, float vx, float vy,
                                     int action, PosFn pos) {
  float ux[NMAX], uy[NMAX];
#pragma unroll
  for (int u = 0; u < NMAX; ++u) pos(u < N ? u : 0, ux[u], uy[u]);   // all reads issued first
  float fx = 0.0f + action_level(action / 3);
  float fy = 0.0f + action_level(action % 3);
  if (scenario == SWARM_OBSTACLE_AVOIDANCE) {
    float gx, gy;
    pair_force(px - kObstX, py - kObstY, gx, gy);
    fx = fx + gx; fy = fy + gy;
  }
#pragma unroll
  for (int u = 0; u < NMAX; ++u) {
    if (u < N) {
      float gx, gy;
      pair_force(px - ux[u], py - uy[u], gx, gy);   // u == agent: dist 0 < 1e-6 -> exactly 0
      fx = fx + gx; fy = fy + gy;
    }
  }
  StepOut o;
  o.vx = vx * kDragKeep;
  o.vy = vy * kDragKeep;
  o.vx = o.vx + (fx / 1.0f) * kDt;
  o.vy = o.vy + (fy / 1.0f) * kDt;
  o.px = px + o.vx * kDt;
  o.py = py + o.vy * kDt;
  o.dgoal = norm2(o.px - kGoalX, o.py - kGoalY);
  o.dobs = (norm2(o.px - kObstX, o.py - kObstY) - kRadius) - kRadius;
  return o;
}

// OA per-agent reward (obstacle_avoidance_scenario.py:283-300)
__device__ inline float oa_reward(float dgoal, float dobs) {
  const float obst = dobs <= 1.0f ? -(1.0f - dobs) : 0.0f;
  return -dgoal + 2.5f * obst;
}

}  // namespace swarm
