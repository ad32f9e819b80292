// swarm_gat3.h — the three-layer GAT (hidden 8) held by the reference's Flocking
// checkpoints (data/models/experiment_Flocking-seed_*.pth: conv1..conv3, lin1, lin2),
// forward only (acting and evaluation), one graph per wave with the D layout's lane map
// (node n = 16 ct + c, row group p).
//
// Architecture: the GCN class with its commented layers (train_gcn_dqn.py:51-70, the
// conv2/conv3 lines :54-55 and :65-68):
//   conv1 -> tanh -> conv2 -> relu -> conv3 -> relu -> lin1 -> relu -> lin2
// GATConv math as in swarm_dl.h (PyG 2.5.3, heads 1, no added self loops, duplicate
// edges counted by multiplicity).  Hidden 8 is narrower than an MFMA tile, so the products
// are per-node VALU dot products: row group p owns features 2p and 2p + 1, and node rows
// (layer inputs, conv outputs) go through the wave's private LDS rows with wave syncs.
#pragma once
#include "swarm_dl.h"

namespace swarm {

constexpr int kH3 = 8;
// flat layout == the checkpoint's state_dict order; inside a conv: att_src, att_dst, bias,
// lin.weight [8][K] (K = 7 for conv1, 8 after)
__host__ __device__ constexpr int g3_conv_off(int l) { return l == 0 ? 0 : 80 + 88 * (l - 1); }
constexpr int G3_ATT_SRC = 0, G3_ATT_DST = 8, G3_BIAS = 16, G3_W = 24;
constexpr int G3_LIN1_W = 256, G3_LIN1_B = 320, G3_LIN2_W = 328, G3_LIN2_B = 400;
constexpr int G3_N_PARAMS = 409;
static_assert(g3_conv_off(2) + G3_W + kH3 * kH3 == G3_LIN1_W, "gat3 layout");
static_assert(G3_N_PARAMS <= N_LDS_PARAMS, "gat3 weights fit the acting LDS image");

// the first 8 floats of an LDS row (rows are 16-B aligned: kRow = 36)
__device__ inline void load_row8(const float* row, float x[kH3]) {
  const float4 a = *reinterpret_cast<const float4*>(row);
  const float4 b = *reinterpret_cast<const float4*>(row + 4);
  x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w; x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
}

// Fills F.q (and sm.Q, sm.px / sm.py, the graph masks of sm) like dl_forward; P holds the
// 409 weights unpadded.  F.x must hold the lane's features (zero for nodes >= N).
template <int NS>
__device__ inline void gat3_forward(const float* __restrict__ P, const DGeom<NS>& d, int N, int graph, int k,
                                    float radius, const uint8_t* __restrict__ dense, const WView<NS>& V,
                                    DFwd<NS>& F) {
  constexpr int CT = DGeom<NS>::CT;
  WSmall<NS>& sm = *V.sm;
  const int c = d.c, p = d.p;
  // layer-1 input rows X[n][0..7] = (px py vx vy gx gy id 0) in V.H; positions for the graph
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    const int n = 16 * ct + c;
    if (n < NS) {
      V.H[n][p] = F.x[ct][0];
      V.H[n][4 + p] = F.x[ct][1];
      if (p == 0) sm.px[n] = F.x[ct][0];
      if (p == 1) sm.py[n] = F.x[ct][0];
    }
  }
  wave_lds_sync();
  // neighbour masks (dl_forward's graph phase; T / R rows are free scratch until layer 1)
  if (graph == SWARM_GRAPH_KNN) {
    if constexpr (NS <= 16) {
      knn_masks_wave<NS, NS>(d.lane, N, k, sm, &V.T[0][0], reinterpret_cast<KV*>(&V.R[0][0]), V.memo);
    } else {
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        const int n = 16 * ct + c;
        KV* q = reinterpret_cast<KV*>(&V.T[0][0]) + (n < NS ? n : 0) * NS;
        if (n < NS && p == 0) sm.knn[n] = (n < N) ? knn_mask_node<NS, NS>(n, N, k, sm, q) : 0u;
      }
    }
    wave_lds_sync();
  } else if (graph == SWARM_GRAPH_RADIUS) {
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      const int n = 16 * ct + c;
      if (n < NS && p == 0) sm.knn[n] = radius_mask_node<NS, NS>(n, N, radius, sm);
    }
    wave_lds_sync();
  }
  // in-edge multiplicities of the lane's node: the same graph for all three layers
  constexpr bool kKeepM = NS <= 16;   // registers: NS ints per column tile
  int mk[kKeepM ? CT : 1][kKeepM ? NS : 1];
  if constexpr (kKeepM) {
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) in_mults<NS>(min(16 * ct + c, NS - 1), N, graph, sm, dense, d.gid, mk[ct]);
  }
#pragma unroll
  for (int l = 0; l < 3; ++l) {
    const float* Pc = P + g3_conv_off(l);
    const int K = l == 0 ? kFeat : kH3;
    // ---- lin: h[n][2p + i] = sum_k W[2p + i][k] X[n][k]; scores reduced over the row groups
    float h[CT][2], sdst[CT];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      const int n = min(16 * ct + c, NS - 1);
      float x[kH3];
      load_row8(&V.H[n][0], x);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const float* w = Pc + G3_W + (2 * p + i) * K;
        float acc = 0.0f;
#pragma unroll
        for (int kk = 0; kk < kH3; ++kk)
          if (kk < K) acc = acc + w[kk] * x[kk];
        h[ct][i] = acc;
      }
      const float ps = h[ct][0] * Pc[G3_ATT_SRC + 2 * p] + h[ct][1] * Pc[G3_ATT_SRC + 2 * p + 1];
      const float pd = h[ct][0] * Pc[G3_ATT_DST + 2 * p] + h[ct][1] * Pc[G3_ATT_DST + 2 * p + 1];
      const float ss = row4_sum(ps);
      sdst[ct] = row4_sum(pd);
      const int nn = 16 * ct + c;
      if (nn < NS) {
        *reinterpret_cast<float2*>(&V.T[nn][2 * p]) = make_float2(h[ct][0], h[ct][1]);
        if (p == 0) sm.ssrc[nn] = ss;
      }
    }
    wave_lds_sync();
    // ---- attention softmax over n's in-edges and the aggregation, + bias, activation
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      const int n = 16 * ct + c;
      int m[NS];
      if constexpr (kKeepM) {
#pragma unroll
        for (int u = 0; u < NS; ++u) m[u] = mk[ct][u];
      } else {
        in_mults<NS>(min(n, NS - 1), N, graph, sm, dense, d.gid, m);
      }
      float e[NS];
      float emax = -INFINITY;
#pragma unroll
      for (int u = 0; u < NS; ++u) {
        e[u] = leaky(sm.ssrc[u] + sdst[ct]);
        emax = m[u] > 0 ? fmaxf(emax, e[u]) : emax;
      }
      float den = 0.0f;
#pragma unroll
      for (int u = 0; u < NS; ++u) {
        e[u] = m[u] > 0 ? __expf(e[u] - emax) : 0.0f;
        den = den + (float)m[u] * e[u];
      }
      const float inv = 1.0f / (den + 1e-16f);
      float o0 = 0.0f, o1 = 0.0f;
#pragma unroll
      for (int u = 0; u < NS; ++u) {
        const float cf = (float)m[u] * (e[u] * inv);
        const float2 hu = *reinterpret_cast<const float2*>(&V.T[u][2 * p]);
        o0 = o0 + cf * hu.x;
        o1 = o1 + cf * hu.y;
      }
      o0 = o0 + Pc[G3_BIAS + 2 * p];
      o1 = o1 + Pc[G3_BIAS + 2 * p + 1];
      if (l == 0) { o0 = tanh_fast(o0); o1 = tanh_fast(o1); }
      else { o0 = o0 > 0.0f ? o0 : 0.0f; o1 = o1 > 0.0f ? o1 : 0.0f; }
      if (n < NS) *reinterpret_cast<float2*>(&V.H[n][2 * p]) = make_float2(o0, o1);   // next layer's input row
    }
    wave_lds_sync();
  }
  // ---- lin1 + relu (rows to V.R), then lin2 (Q rows to sm.Q)
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    const int n = min(16 * ct + c, NS - 1);
    float x[kH3];
    load_row8(&V.H[n][0], x);
    float z[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const float* w = P + G3_LIN1_W + (2 * p + i) * kH3;
      float acc = 0.0f;
#pragma unroll
      for (int kk = 0; kk < kH3; ++kk) acc = acc + w[kk] * x[kk];
      acc = acc + P[G3_LIN1_B + 2 * p + i];
      z[i] = acc > 0.0f ? acc : 0.0f;
    }
    if (16 * ct + c < NS) *reinterpret_cast<float2*>(&V.R[n][2 * p]) = make_float2(z[0], z[1]);
  }
  wave_lds_sync();
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    const int n = min(16 * ct + c, NS - 1);
    float z[kH3];
    load_row8(&V.R[n][0], z);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int a = p + 4 * j;
      if (a < kActions && 16 * ct + c < NS) {
        const float* w = P + G3_LIN2_W + a * kH3;
        float acc = 0.0f;
#pragma unroll
        for (int kk = 0; kk < kH3; ++kk) acc = acc + w[kk] * z[kk];
        sm.Q[n][a] = acc + P[G3_LIN2_B + a];
      }
    }
  }
  wave_lds_sync();
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    const int n = min(16 * ct + c, NS - 1);
#pragma unroll
    for (int a = 0; a < kActions; ++a) F.q[ct][a] = sm.Q[n][a];
  }
}

}  // namespace swarm
