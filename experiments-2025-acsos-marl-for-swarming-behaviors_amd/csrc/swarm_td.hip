// swarm_td.hip — learning side of the hot path: replay sample, TD loss, hand-written
// backward through GCN (PyG GATConv + MLP), deterministic gradient reduction,
// clip_grad_norm_ and Adam.  gfx950 only.
//
// Reference: DQNTrainer.train_step_dqn (src/training/train_gcn_dqn.py:112-137),
// GraphReplayBuffer.sample (:38-45), Adam(lr=1e-3) (:85), target sync (:131-133).
//
// Layout (swarm_wpg.h): one wave per sampled graph; a block holds 32 node slots.
// Backward per graph (online wave, per-node vectors in registers):
//   dQ[a] = (Q[a]-y) * 2/M                      (MSELoss mean, gather)
//   dR = W2[a]^T dQ ; dZ = dR * [Z>0] ; dT = W1^T dZ ; dOut = dT * (1 - t^2)
//   GAT: g_uv = dOut_v.h_u ; de_uv = c_uv (g_uv - sum_w c_wv g_wv) ; dp = de * leaky'(p)
//        da_dst[v] = sum_u dp_uv ; da_src[u] = sum_v dp_uv ; dh_u = sum_v c_uv dOut_v + da_src att_src + da_dst att_dst
// Parameter sums over the block's 32 node rows: dW1 = dZ^T T, dW2 = dQ^T R, dW = dh^T X on
// MFMA (32x32x2 f32, node index as K), vectors by LDS column sums; each block writes one
// slab [N_PARAMS + 1] (last = sum of squared TD errors) and swarm_grad_reduce sums the
// slabs in a fixed order (bitwise run-to-run reproducible).
#include <stdlib.h>

#include "swarm_adam.h"
#include "swarm_dl.h"

namespace swarm {

// One TD block = 32 node slots = GPB = 32 / NS sampled graphs.  Wave w < GPB runs the
// ONLINE network on graph w (forward on s with activations kept, dQ, backward of the
// per-node vectors); wave GPB + w runs the TARGET network on s' of graph w
// (y = r + gamma max_a Q_tgt), then shares the parameter products.  The parameter
// gradient of the block is a sum over its 32 node rows: MFMA 32x32x2 f32 with the
// node index as K, jobs spread over the waves, each writing its slice of the slab.
constexpr int kTdRows = 32;

template <int NS>
struct TdLds {
  static constexpr int GPB = kTdRows / NS;
  float H[kTdRows][kRow];         // online conv1.lin output
  float T[kTdRows][kRow];         // tanh(conv out)
  float R[kTdRows][kRow];         // relu(lin1)
  float dZ[kTdRows][kRow];        // dL/d lin1 pre-activation
  float dO[kTdRows][kRow];        // dL/d conv out
  float dH[kTdRows][kRow];        // dL/d h
  float X[kTdRows][9];            // node features (k < 8)
  float cm[kTdRows][NS + 1];      // c[target row][source slot]
  float dp[kTdRows][NS + 1];      // dL/d pre-activation of edge (source -> target row)
  float y[kTdRows], gq[kTdRows], das[kTdRows], dad[kTdRows], d2[kTdRows];
  int act[kTdRows];
  WSmall<NS> on[GPB];             // online waves' per-graph scratch
  WScratch<NS> tg[GPB];           // target waves' forward scratch
};

struct TdArgs {
  int S, B, N, graph, k, conv, env_offset;
  uint32_t k0, k1;
  const float* params;
  const float* target;
  swarm_replay replay;
  const swarm_ctrl* ctrl;
  const int32_t* sample_in;
  int32_t* sample_out;
  float* slabs;
  float gamma;
  float grad_scale;   // fp32(2 / M_local)
};

// gradient-slab store (read once by the next launch, from another XCD).  Plain stores:
// measured against nt (1: td 8.4 vs 8.0 us) and write-through sc1 (2: 9.5 us) stores.
__device__ inline void slab_st(float* p, float v) {
#if SWARM_SLAB_ST == 1
  __builtin_nontemporal_store(v, p);
#elif SWARM_SLAB_ST == 2
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // write-through (sc1)
#else
  *p = v;
#endif
}

// D[i][j] = sum_node A_img[node][i] * B_img[node][j] over the 32 node rows (MFMA, K = node)
__device__ inline f32x16 mfma_nodesum(const float (*Aimg)[kRow], const float (*Bimg)[kRow], int lane) {
  f32x16 acc = {};
  const int h = lane >> 5, c = lane & 31;
#pragma unroll
  for (int s = 0; s < 16; ++s) acc = mfma32(Aimg[2 * s + h][c], Bimg[2 * s + h][c], acc);
  return acc;
}

// NS node slots per wave holding NS / GS graphs of GS slots (GS = 8 < NS = 16 packs two
// N <= 8 graphs into one wave: every MFMA column is a real node, one wave per SIMD).
// The dependent chain's pointers (batch indices -> replay rows) and the geometry lead the
// parameter list: preloaded into SGPRs (kernarg preload), the index loads issue at wave start.
template <int NS, int GS, int SPEC>   // SPEC: graph + conv fixed at compile time (swarm_common.h)
__global__ __launch_bounds__(128 * (kTdRows / NS)) void td_kernel(const int32_t* sample_in, const float* rs, const float* rs_next,
                                                                       const float* rr, const uint8_t* ra, int S, int B, int N,
                                                                       int capacity, TdArgs A) {
  constexpr int GPB = kTdRows / NS, CT = DGeom<NS>::CT;   // GPB: online (= target) waves per block
  constexpr int GPW = NS / GS;                             // graphs per wave
  constexpr int NT = 128 * GPB;
  __shared__ TdLds<NS> TB;
  __shared__ __attribute__((aligned(16))) float Pon[N_LDS_PARAMS];
  __shared__ __attribute__((aligned(16))) float Ptg[N_LDS_PARAMS];
  const int wave = threadIdx.x >> 6;
  const bool online = wave < GPB;
  const int wi = online ? wave : wave - GPB;
  const DGeom<NS> d = make_dgeom<NS>(blockIdx.x * GPB + wi, 1 << 30);   // lane geometry; liveness is per graph
  const int graph = spec_graph<SPEC>(A.graph);
  const int conv = spec_conv<SPEC>(A.conv);
  const int row0 = wi * NS;
  const WView<NS> V = online ? WView<NS>{TB.H + row0, TB.T + row0, TB.R + row0, &TB.on[wi]} : TB.tg[wi].view();
  const int lane = d.lane, c = d.c, p = d.p;
  float* gslab = A.slabs + (size_t)blockIdx.x * (N_PARAMS + 1);
  SWARM_RTSTAMP(8);
  SWARM_STAMP(0);

  // ---- fused tick: this wave's replay indices come from the previous launch, so the
  //      dependent pair (index -> replay rows) is issued first and the weight staging and
  //      ctrl reads overlap it.  Indices are clamped into the ring: a skipped tick reads
  //      valid (unused) rows.
  const uint32_t cap = (uint32_t)capacity;
  const uint32_t ring_graphs = cap * (uint32_t)B;
  int sid[CT];     // batch index of this lane's graph
  bool live[CT], nv[CT];
  int jl[CT];      // local node index inside the graph
  uint32_t gid[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    const int n = 16 * ct + c;
    const int gi = (GS < NS) ? n / GS : 0;
    jl[ct] = (GS < NS) ? n % GS : n;
    sid[ct] = blockIdx.x * (kTdRows / GS) + wi * GPW + gi;
    live[ct] = sid[ct] < S && n < NS;
    nv[ct] = live[ct] && jl[ct] < N;
    gid[ct] = 0;
    if (sample_in) gid[ct] = min((uint32_t)sample_in[min(sid[ct], S - 1)], ring_graphs - 1u);
  }
  ParamStage<NT> pon, ptg;
  pon.load(A.params, threadIdx.x);
  ptg.load(A.target, threadIdx.x);
  const uint32_t filled = A.ctrl->filled_slots;
  const uint32_t valid_slots = filled + 1 < cap ? filled + 1 : cap;
  const uint32_t n_graphs = valid_slots * (uint32_t)B;
  if (!sample_in) {   // GraphReplayBuffer.sample: random.sample -> keyed permutation
    const SampleKey sk = sample_key(n_graphs, A.k0 ^ ((uint32_t)A.env_offset * 0x9E3779B9u), A.k1, A.ctrl->tick);
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
      gid[ct] = n_graphs >= (uint32_t)S ? sample_index((uint32_t)min(sid[ct], S - 1), sk) : 0u;
  }
  float rew[CT];
  int act[CT];
  DFwd<NS> F;
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    const uint32_t slot = gid[ct] / (uint32_t)B, genv = gid[ct] % (uint32_t)B;
    const size_t ri = ((size_t)slot * B + genv) * N + min(jl[ct], N - 1);
    const float4 st = reinterpret_cast<const float4*>(online ? rs : rs_next)[ri];
    rew[ct] = rr[ri];
    act[ct] = nv[ct] ? (int)ra[ri] : 0;
    node_x(st.x, st.y, st.z, st.w, jl[ct], p, F.x[ct]);
    if (!nv[ct]) { F.x[ct][0] = 0.0f; F.x[ct][1] = 0.0f; }
  }
  // ---- skip while the replay holds fewer than `batch` graphs (train_gcn_dqn.py:113-115)
  if (n_graphs < (uint32_t)S) {
    for (int q = threadIdx.x; q <= N_PARAMS; q += NT) slab_st(gslab + (q), 0.0f);
    return;
  }
  if (A.sample_out && online && p == 0) {
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
      if (live[ct] && jl[ct] == 0) A.sample_out[sid[ct]] = (int32_t)gid[ct];
  }
  SWARM_STAMP(1);
  pon.store(Pon, threadIdx.x);
  ptg.store(Ptg, threadIdx.x);
  if (online && p == 0) {
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
      if (16 * ct + c < NS) TB.act[row0 + 16 * ct + c] = act[ct];
  }
  __syncthreads();   // B0: weight images
  SWARM_STAMP(2);
  // ---- forwards: online on s (activations kept), target on s' (train_gcn_dqn.py:119-121).
  //      Everything after B1 waits for the target waves' y, so they issue first.
  if (!online) __builtin_amdgcn_s_setprio(2);
  dl_forward<NS, 16, GS>(online ? Pon : Ptg, d, N, graph, A.k, conv, nullptr, V, online, F);
  if (!online && p == 0) {
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      float qmax = F.q[ct][0];
#pragma unroll
      for (int a = 1; a < kActions; ++a) qmax = fmaxf(qmax, F.q[ct][a]);
      if (16 * ct + c < NS) TB.y[row0 + 16 * ct + c] = nv[ct] ? rew[ct] + A.gamma * qmax : 0.0f;
    }
  }
  if (!online) __builtin_amdgcn_s_setprio(0);
  SWARM_STAMP(3);
  __syncthreads();   // B1: TD targets
  SWARM_STAMP(4);

  const float* P = Pon;
  float dz[CT][2][4];
  if (online) {
    // ---- dQ at the taken action (MSELoss mean), dR = W2[a]^T dQ, dZ = dR * [z > 0]
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      const int n = 16 * ct + c, nn = min(n, NS - 1);
      float qa = F.q[ct][0];
#pragma unroll
      for (int a = 1; a < kActions; ++a) qa = (act[ct] == a) ? F.q[ct][a] : qa;
      const float delta = nv[ct] ? (qa - TB.y[row0 + nn]) : 0.0f;
      const float gq = delta * A.grad_scale;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const float4 w = *reinterpret_cast<const float4*>(P + L_W2 + act[ct] * kWRow + 16 * t + 4 * p);
        const float wv[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int r = 0; r < 4; ++r) dz[ct][t][r] = F.zr[ct][t][r] > 0.0f ? wv[r] * gq : 0.0f;
      }
      if (n < NS) {
        const int row = row0 + n;
        *reinterpret_cast<float4*>(&TB.dZ[row][4 * p]) = make_float4(dz[ct][0][0], dz[ct][0][1], dz[ct][0][2], dz[ct][0][3]);
        *reinterpret_cast<float4*>(&TB.dZ[row][16 + 4 * p]) = make_float4(dz[ct][1][0], dz[ct][1][1], dz[ct][1][2], dz[ct][1][3]);
        TB.X[row][p] = F.x[ct][0];
        TB.X[row][4 + p] = F.x[ct][1];
#pragma unroll
        for (int j = 0; j < NS / 4; ++j) TB.cm[row][4 * j + p] = pick4(F.cf[ct], j, p);
        if (p == 0) { TB.X[row][8] = 0.0f; TB.gq[row] = gq; TB.d2[row] = delta * delta; }
      }
    }
  }
  __syncthreads();   // B2: dZ / T / R / gq / act / d2 / X / cm of every graph
  SWARM_STAMP(5);

  const int col = lane & 31, h = lane >> 5;
  if (online) {
    // ---- dT^T = W1^T dZ^T on MFMA (the dz registers are the B operand),
    //      dO = dT * (1 - t^2) with the forward's tanh registers
    float dO[CT][2][4];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      const int n = 16 * ct + c;
#pragma unroll
      for (int t2 = 0; t2 < 2; ++t2) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            acc = mfma16(P[L_W1 + (16 * t + 4 * p + r) * kWRow + 16 * t2 + c], dz[ct][t][r], acc);
#pragma unroll
        for (int r = 0; r < 4; ++r)
          dO[ct][t2][r] = nv[ct] ? acc[r] * (1.0f - F.t[ct][t2][r] * F.t[ct][t2][r]) : 0.0f;
      }
      if (n < NS) {
        *reinterpret_cast<float4*>(&TB.dO[row0 + n][4 * p]) = make_float4(dO[ct][0][0], dO[ct][0][1], dO[ct][0][2], dO[ct][0][3]);
        *reinterpret_cast<float4*>(&TB.dO[row0 + n][16 + 4 * p]) = make_float4(dO[ct][1][0], dO[ct][1][1], dO[ct][1][2], dO[ct][1][3]);
      }
    }
    SWARM_STAMP(24);
    // ---- GAT backward (attention part).  g[u][v] = H_u . dO_v on MFMA (A = H rows,
    //      B = the dO registers); lane (c, p) holds g[u = 16 ut + 4 p + r][v = 16 ct + c]
    float da_d[CT];
    WSmall<NS>& sm = *V.sm;
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) da_d[ct] = 0.0f;
    if (conv == SWARM_CONV_GAT) {
      float ah[CT][2][4];
#pragma unroll
      for (int ut = 0; ut < CT; ++ut) {
        const int u = min(16 * ut + c, NS - 1);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const float4 hv = *reinterpret_cast<const float4*>(&TB.H[row0 + u][16 * t + 4 * p]);
          ah[ut][t][0] = hv.x; ah[ut][t][1] = hv.y; ah[ut][t][2] = hv.z; ah[ut][t][3] = hv.w;
        }
      }
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        const int v = 16 * ct + c;
        float gv[CT][4], cu[CT][4];
        float part = 0.0f;
#pragma unroll
        for (int ut = 0; ut < CT; ++ut) {
          f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc = mfma16(ah[ut][t][r], dO[ct][t][r], acc);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            // coefficient of edge u -> v, u = 16 ut + 4 p + r (registers hold every u of target v)
            float cc[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int uq = 16 * ut + 4 * q + r;
              cc[q] = uq < NS ? F.cf[ct][uq < NS ? uq : 0] : 0.0f;
            }
            cu[ut][r] = p == 0 ? cc[0] : (p == 1 ? cc[1] : (p == 2 ? cc[2] : cc[3]));
            gv[ut][r] = acc[r];
            part = part + cu[ut][r] * gv[ut][r];
          }
        }
        const float Gs = row4_sum(part);
        float dsum = 0.0f;
#pragma unroll
        for (int ut = 0; ut < CT; ++ut)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int u = 16 * ut + 4 * p + r;
            float dpu = 0.0f;
            if (u < NS && cu[ut][r] != 0.0f && nv[ct]) {   // in-edges only (cross-graph / absent: c = 0)
              const float de = cu[ut][r] * (gv[ut][r] - Gs);
              const float pre = sm.ssrc[u] + F.sdst[ct];
              dpu = pre > 0.0f ? de : de * kLeakySlope;
            }
            dsum = dsum + dpu;
            if (u < NS && v < NS) TB.dp[row0 + v][u] = dpu;
          }
        da_d[ct] = row4_sum(dsum);
      }
    }
    wave_lds_sync();   // dp / dO rows of this graph
    SWARM_STAMP(25);
    // ---- dh_u = sum_v c[v][u] dO_v (MFMA: A = dO rows, B = C column) + da_src att_src + da_dst att_dst
    const float4 s0 = *reinterpret_cast<const float4*>(P + L_ATT_SRC + 4 * p);
    const float4 s1 = *reinterpret_cast<const float4*>(P + L_ATT_SRC + 16 + 4 * p);
    const float4 d0 = *reinterpret_cast<const float4*>(P + L_ATT_DST + 4 * p);
    const float4 d1 = *reinterpret_cast<const float4*>(P + L_ATT_DST + 16 + 4 * p);
    const float as[2][4] = {{s0.x, s0.y, s0.z, s0.w}, {s1.x, s1.y, s1.z, s1.w}};
    const float ad[2][4] = {{d0.x, d0.y, d0.z, d0.w}, {d1.x, d1.y, d1.z, d1.w}};
    float ao[2][NS / 4];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int ks = 0; ks < NS / 4; ++ks) ao[t][ks] = TB.dO[row0 + 4 * ks + p][16 * t + c];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      const int u = 16 * ct + c, uu = min(u, NS - 1);
      float da_s = 0.0f;
      if (conv == SWARM_CONV_GAT) {   // sum over the targets v of u's own graph
        const int base = (GS < NS) ? (uu / GS) * GS : 0;
#pragma unroll
        for (int j = 0; j < GS; ++j)
          if (j < N) da_s = da_s + TB.dp[row0 + base + j][uu];
      }
      const float das = nv[ct] ? da_s : 0.0f, dad = nv[ct] ? da_d[ct] : 0.0f;
      f32x4 m0 = {0.f, 0.f, 0.f, 0.f}, m1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < NS / 4; ++ks) {
        const float b = TB.cm[row0 + 4 * ks + p][uu];
        m0 = mfma16(ao[0][ks], b, m0);
        m1 = mfma16(ao[1][ks], b, m1);
      }
      float dh[2][4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        dh[0][r] = nv[ct] ? (m0[r] + das * as[0][r]) + dad * ad[0][r] : 0.0f;
        dh[1][r] = nv[ct] ? (m1[r] + das * as[1][r]) + dad * ad[1][r] : 0.0f;
      }
      if (u < NS) {
        *reinterpret_cast<float4*>(&TB.dH[row0 + u][4 * p]) = make_float4(dh[0][0], dh[0][1], dh[0][2], dh[0][3]);
        *reinterpret_cast<float4*>(&TB.dH[row0 + u][16 + 4 * p]) = make_float4(dh[1][0], dh[1][1], dh[1][2], dh[1][3]);
        if (p == 0) { TB.das[row0 + u] = das; TB.dad[row0 + u] = dad; }
      }
    }
    SWARM_STAMP(27);
  } else {
    // ---- target waves: products that need only B2's images
    //      job 0: dW1 = dZ^T T ; job 1: dW2 = onehot(a) gq R, db2, loss ; job 2: db1
    for (int job = wi; job < 3; job += GPB) {
      if (job == 0) {
        const f32x16 dW1 = mfma_nodesum(TB.dZ, TB.T, lane);
#pragma unroll
        for (int r = 0; r < 16; ++r) slab_st(gslab + (OFF_W1 + acc_row(r, h) * kHidden + col), dW1[r]);
      } else if (job == 1) {
        f32x16 dW2 = {};
#pragma unroll
        for (int s = 0; s < 16; ++s) {
          const int n = 2 * s + h;
          const float a = (TB.act[n] == col) ? TB.gq[n] : 0.0f;
          dW2 = mfma32(a, TB.R[n][col], dW2);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int a = acc_row(r, h);
          if (a < kActions) slab_st(gslab + (OFF_W2 + a * kHidden + col), dW2[r]);
        }
        if (lane < kActions || lane == 63) {   // every read issued before the ordered sum
          float v[kTdRows];
#pragma unroll
          for (int n = 0; n < kTdRows; ++n) v[n] = lane == 63 ? TB.d2[n] : (TB.act[n] == lane ? TB.gq[n] : 0.0f);
          float acc = v[0];
#pragma unroll
          for (int n = 1; n < kTdRows; ++n) acc = acc + v[n];
          slab_st(gslab + (lane == 63 ? N_PARAMS : OFF_B2 + lane), acc);
        }
      } else {
        if (lane < kHidden) {
          float v[kTdRows];
#pragma unroll
          for (int n = 0; n < kTdRows; ++n) v[n] = TB.dZ[n][lane];
          float acc = v[0];
#pragma unroll
          for (int n = 1; n < kTdRows; ++n) acc = acc + v[n];
          slab_st(gslab + (OFF_B1 + lane), acc);
        }
      }
    }
  }
  __syncthreads();   // B3: dO / dH / das / dad
  SWARM_STAMP(6);
  // ---- products over B3's images, spread over all 2 GPB waves of the block:
  //      job 0 / 1: dW rows 0-15 / 16-31 = sum_n dH[n][f] X[n][k] (MFMA 16x16x4, K = node rows)
  //      job 2: att_src / att_dst (lane halves) ; job 3: dbias
  {
    const int wall = online ? wi : GPB + wi;
    for (int job = wall; job < 4; job += 2 * GPB) {
      if (job < 2) {
        const int t = job;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < kTdRows / 4; ++ks) {
          const int n = 4 * ks + p;
          acc = mfma16(TB.dH[n][16 * t + c], c < kFeat ? TB.X[n][c] : 0.0f, acc);
        }
        if (c < kFeat) {
#pragma unroll
          for (int r = 0; r < 4; ++r) slab_st(gslab + (OFF_W + (16 * t + 4 * p + r) * kFeat + c), acc[r]);
        }
      } else if (job == 2) {   // att_src (half 0) / att_dst (half 1): sum_n da[n] H[n][col]
        const float* da = h == 0 ? TB.das : TB.dad;
        float v[kTdRows];
#pragma unroll
        for (int n = 0; n < kTdRows; ++n) v[n] = da[n] * TB.H[n][col];
        float acc = v[0];
#pragma unroll
        for (int n = 1; n < kTdRows; ++n) acc = acc + v[n];
        slab_st(gslab + ((h == 0 ? OFF_ATT_SRC : OFF_ATT_DST) + col), acc);
      } else if (lane < kHidden) {
        float v[kTdRows];
#pragma unroll
        for (int n = 0; n < kTdRows; ++n) v[n] = TB.dO[n][lane];
        float acc = v[0];
#pragma unroll
        for (int n = 1; n < kTdRows; ++n) acc = acc + v[n];
        slab_st(gslab + (OFF_BIAS + lane), acc);
      }
    }
  }
  SWARM_STAMP(7);
  SWARM_RTSTAMP(9);
}

// ---------------------------------------------------------------- slab reduction
// block = 256 threads covers 64 columns; thread (col, part) sums a contiguous quarter
// of the slabs, quarters combined in order: fixed order -> bitwise reproducible.
struct ReduceArgs {
  int n_slabs;
  const float* slabs;
  float* grad;
  int advance;            // fused tick: copy *_nxt -> *_cur and advance ctrl
  swarm_learner lr;
  swarm_ctrl* ctrl;
  int capacity, B, N, batch;
  swarm_adam_cfg hp;
  uint32_t k0, k1;        // replay-sampling key (seed ^ rank salt)
};

// 1024 threads = 16 columns x 64 slab groups (105 blocks: the 1.7 MB of freshly written
// slabs is read by many CUs at once, 16 KB each); group g sums a contiguous run of slabs
// with every load issued before the ordered adds, then the 64 group sums of a column are
// added in group order (fixed order -> bitwise reproducible run to run).
constexpr int kRedCols = 16;
constexpr int kRedGroups = 64;
// slabs / ctrl / geometry preloaded into SGPRs (kernarg preload): the slab loads issue at wave start
__global__ __launch_bounds__(kRedCols * kRedGroups) void grad_reduce_kernel(const float* slabs, swarm_ctrl* ctrl,
                                                                            int n_slabs, int advance, ReduceArgs A) {
  __shared__ float part[kRedGroups][kRedCols];
  SWARM_RTSTAMP(22);
  SWARM_STAMP(28);
  const int c = threadIdx.x % kRedCols;
  const int col = blockIdx.x * kRedCols + c;
  const int q = threadIdx.x / kRedCols;
  // advance mode: the thread owning column N_PARAMS is the control block's single writer.
  // It reads ctrl and prepares the whole update (incl. the double-precision Adam scalars
  // of the next step) before the slab loads return, and stores it at the end.
  const bool writer = advance && col == N_PARAMS && q == 0;
  const int per = (n_slabs + kRedGroups - 1) / kRedGroups;
  const int b0 = q * per, b1 = min(n_slabs, b0 + per);
  // first chunk of this thread's slab column in flight before anything else
  constexpr int kChunk = 8;
  float v0[kChunk];
#pragma unroll
  for (int j = 0; j < kChunk; ++j)
    v0[j] = (col <= N_PARAMS && b0 + j < b1) ? slabs[(size_t)(b0 + j) * (N_PARAMS + 1) + col] : 0.0f;
  // advance mode: the thread owning column N_PARAMS is the control block's single writer.
  // It prepares the whole update (incl. the double-precision Adam scalars of the next
  // step and the next tick's sampling key) while the slab loads fly, stores it at the end.
  swarm_ctrl* C = ctrl;
  uint32_t c_trained = 0, c_step = 0, c_tick = 0, c_slot = 0, c_filled = 0;
  double b1p = 1.0, b2p = 1.0;
  float next_step_size = 0.0f, next_inv_bc2 = 0.0f;
  SampleKey nk = {};
  uint32_t nk_n = 0, nk_tick = 0;
  if (writer) {
    c_trained = C->trained; c_step = C->adam_step; c_tick = C->tick; c_slot = C->write_slot; c_filled = C->filled_slots;
    b1p = ctrl_get_double(C, CTRL_B1POW);
    b2p = ctrl_get_double(C, CTRL_B2POW);
    if (c_trained) {   // the step this tick's act kernel applied
      b1p = b1p * (double)A.hp.beta1;
      b2p = b2p * (double)A.hp.beta2;
      adam_next_scalars(A.hp, b1p, b2p, next_step_size, next_inv_bc2);
    }
  }
  // a second wave of the same block prepares the next tick's sampling key in parallel
  const bool key_writer = advance && col == N_PARAMS && q == 4;
  if (key_writer) {
    const uint32_t cap = (uint32_t)A.capacity;
    const uint32_t filled = C->filled_slots;
    const uint32_t f1 = filled + 1 < cap ? filled + 1 : cap;   // filled after this tick
    nk_n = (f1 + 1 < cap ? f1 + 1 : cap) * (uint32_t)A.B;       // graphs the next tick samples from
    nk_tick = C->tick + 1;
    nk = sample_key(nk_n, A.k0, A.k1, nk_tick);
  }
  float s = v0[0];
#pragma unroll
  for (int j = 1; j < kChunk; ++j) s = s + v0[j];
  if (col <= N_PARAMS) {
    for (int b = b0 + kChunk; b < b1; b += kChunk) {
      float v[kChunk];
#pragma unroll
      for (int j = 0; j < kChunk; ++j) v[j] = (b + j < b1) ? slabs[(size_t)(b + j) * (N_PARAMS + 1) + col] : 0.0f;
#pragma unroll
      for (int j = 0; j < kChunk; ++j) s = s + v[j];
    }
  }
  if (advance && col < N_PARAMS) {   // ping-pong copy-back, one array per group
    if (q == 0) A.lr.w_cur[col] = A.lr.w_nxt[col];
    else if (q == 1) A.lr.m_cur[col] = A.lr.m_nxt[col];
    else if (q == 2) A.lr.v_cur[col] = A.lr.v_nxt[col];
  }
  SWARM_STAMP(29);
  part[q][c] = s;
  __syncthreads();
  SWARM_STAMP(30);
  if (q == 0 && col <= N_PARAMS) {
    float tot = part[0][c];
#pragma unroll
    for (int gi = 1; gi < kRedGroups; ++gi) tot = tot + part[gi][c];
    A.grad[col] = tot;
    if (writer) {   // record the pending update, advance the tick
      const uint32_t cap = (uint32_t)A.capacity;
      const uint32_t valid_slots = c_filled + 1 < cap ? c_filled + 1 : cap;
      const uint32_t trained = valid_slots * (uint32_t)A.B >= (uint32_t)A.batch ? 1u : 0u;
      if (c_trained) {
        C->adam_step = c_step + 1;
        ctrl_set_double(C, CTRL_B1POW, b1p);
        ctrl_set_double(C, CTRL_B2POW, b2p);
        C->adam_step_size = next_step_size;
        C->adam_inv_bc2 = next_inv_bc2;
      }
      C->trained = trained;
      C->loss = trained ? tot / (float)((size_t)A.batch * A.N) : 0.0f;
      C->tick = c_tick + 1;
      C->write_slot = (c_slot + 1) % cap;
      C->filled_slots = valid_slots;
    }
  }
  if (key_writer) {   // after the barrier: every thread of the block has read ctrl
    C->sample_key[0] = nk.rk[0]; C->sample_key[1] = nk.rk[1]; C->sample_key[2] = nk.rk[2]; C->sample_key[3] = nk.rk[3];
    C->sample_bits = (uint32_t)nk.bits;
    C->sample_n = nk_n;
    C->sample_tick = nk_tick;
  }
  SWARM_STAMP(31);
  SWARM_RTSTAMP(23);
}

// ---------------------------------------------------------------- clip + Adam + target sync
// Unfused path (swarm_adam_step): apply now, then advance ctrl.  Flush path
// (swarm_adam_flush): apply a pending fused update in place, no advance.
struct AdamArgs {
  swarm_adam_cfg hp;
  int B, N, capacity, flush;
  float* params;
  float* target;
  float* m;
  float* v;
  const float* grad;
  swarm_ctrl* ctrl;
};

__global__ __launch_bounds__(kAdamNT) void adam_kernel(AdamArgs A) {
  __shared__ float red[8 * (kAdamNT / 64) + 8];
  const int tid = threadIdx.x;
  AdamRegs R;
  R.load(A.grad, A.params, A.m, A.v, tid);
  const float loss_sum = A.grad[N_PARAMS];
  swarm_ctrl* C = A.ctrl;
  const uint32_t cap = (uint32_t)A.capacity;
  const uint32_t filled = C->filled_slots;
  const uint32_t valid_slots = filled + 1 < cap ? filled + 1 : cap;
  const uint32_t tick = C->tick;
  const uint32_t step = C->adam_step + 1;
  const float step_size = C->adam_step_size, inv_bc2 = C->adam_inv_bc2;
  const bool train = A.flush ? (C->trained != 0u) : (valid_slots * (uint32_t)A.B >= (uint32_t)A.hp.batch);
  // target sync: unfused = after the TD step of tick `tick` ((tick+1) % every); flush = the
  // fused tick already advanced ctrl, so the pending update belongs to tick - 1
  const bool sync = ((A.flush ? tick : tick + 1) % (uint32_t)A.hp.update_target_every) == 0u;
  __syncthreads();   // every thread has read ctrl before thread 0 rewrites it
  float gn = 0.0f;
  if (train) {
    gn = adam_apply(R, A.hp, step_size, inv_bc2, tid, red);
    store4(A.params, R.w, R.wt, tid);
    store4(A.m, R.m, R.mt, tid);
    store4(A.v, R.v, R.vt, tid);
    if (sync) store4(A.target, R.w, R.wt, tid);
  }
  if (tid == 0) {
    if (train) {
      C->adam_step = step;
      C->grad_norm = gn;
      ctrl_set_double(C, CTRL_B1POW, ctrl_get_double(C, CTRL_B1POW) * (double)A.hp.beta1);
      ctrl_set_double(C, CTRL_B2POW, ctrl_get_double(C, CTRL_B2POW) * (double)A.hp.beta2);
      ctrl_store_next_scalars(C, A.hp);
    }
    if (A.flush) {
      C->trained = 0u;
    } else {
      C->trained = 0u;   // applied now: nothing pending
      C->loss = train ? loss_sum / (float)((size_t)A.hp.batch * A.N) / (float)A.hp.world_size : 0.0f;
      if (!train) C->grad_norm = 0.0f;
      C->tick = tick + 1;
      C->write_slot = (C->write_slot + 1) % cap;
      C->filled_slots = valid_slots;
    }
  }
}

__global__ void ctrl_init_kernel(swarm_adam_cfg hp, float eps, swarm_ctrl* C) {
  uint32_t* w = reinterpret_cast<uint32_t*>(C);
  for (int i = 0; i < (int)(sizeof(swarm_ctrl) / 4); ++i) w[i] = 0u;
  C->eps = eps;
  C->sample_tick = 0xFFFFFFFFu;   // empty sampling-key cache
  ctrl_set_double(C, CTRL_B1POW, 1.0);
  ctrl_set_double(C, CTRL_B2POW, 1.0);
  ctrl_store_next_scalars(C, hp);
}

__global__ void ctrl_advance_kernel(swarm_ctrl* C, int capacity) {
  const uint32_t cap = (uint32_t)(capacity > 0 ? capacity : 1);
  C->tick = C->tick + 1;
  C->write_slot = (C->write_slot + 1) % cap;
  C->filled_slots = C->filled_slots + 1 < cap ? C->filled_slots + 1 : cap;
}

}  // namespace swarm

using namespace swarm;

namespace {
int td_slots(int N) { return N <= 8 ? 8 : (N <= 16 ? 16 : 32); }
// one block per 32 node slots = 32 / NS sampled graphs
int td_blocks(const swarm_config* cfg, int batch) {
  const int gpb = kTdRows / td_slots(cfg->n_agents);
  return (batch + gpb - 1) / gpb;
}
int td_max_blocks(const swarm_config* cfg, int batch) { return td_blocks(cfg, batch); }
}  // namespace
namespace {
int check_td(const swarm_config* c, const swarm_adam_cfg* hp) {
  if (!c || !hp || c->n_agents < 1 || c->n_agents > 32 || c->n_envs < 1 || hp->batch < 1) return SWARM_E_BADARG;
  if (c->graph == SWARM_GRAPH_DENSE) return SWARM_E_BADARG;
  if (c->graph == SWARM_GRAPH_KNN && (c->knn_k < 1 || c->knn_k > c->n_agents)) return SWARM_E_KNN_K;
  if (hp->world_size < 1 || hp->update_target_every < 1) return SWARM_E_BADARG;
  return 0;
}
}  // namespace

extern "C" {

int64_t swarm_td_workspace_floats(const swarm_config* cfg, int32_t batch) {
  if (!cfg || cfg->n_agents < 1 || cfg->n_agents > 32 || batch < 1) return SWARM_E_BADARG;
  return (int64_t)td_max_blocks(cfg, batch) * (N_PARAMS + 1);
}

int swarm_td_grad(const swarm_config* cfg, const swarm_adam_cfg* hp, const float* params, const float* target,
                  const swarm_replay* replay, const swarm_ctrl* ctrl, const int32_t* sample_in, int32_t* sample_out,
                  float* slabs, void* stream) {
  if (int e = check_td(cfg, hp)) return e;
  if (!replay || !ctrl || !slabs || replay->capacity < 1) return SWARM_E_BADARG;
  TdArgs a = {};
  a.S = hp->batch; a.B = cfg->n_envs; a.N = cfg->n_agents; a.graph = cfg->graph; a.k = cfg->knn_k;
  a.conv = cfg->conv; a.env_offset = cfg->env_offset;
  a.k0 = (uint32_t)(cfg->seed & 0xFFFFFFFFu); a.k1 = (uint32_t)(cfg->seed >> 32);
  a.params = params; a.target = target; a.replay = *replay; a.ctrl = ctrl;
  a.sample_in = sample_in; a.sample_out = sample_out; a.slabs = slabs;
  a.gamma = hp->gamma;
  a.grad_scale = (float)(2.0 / ((double)hp->batch * (double)cfg->n_agents));
  const int nb = td_blocks(cfg, hp->batch);
  hipStream_t st = (hipStream_t)stream;
  const int spec = spec_of(a.graph, a.conv);   // training graphs are complete: GAT and GCN specialised
#define SWARM_TD_LAUNCH1(NS, GS, NT, SP)                                                                       \
  hipLaunchKernelGGL((td_kernel<NS, GS, SP>), dim3(nb), dim3(NT), 0, st, a.sample_in, a.replay.s, a.replay.s_next, \
                     a.replay.r, a.replay.a, a.S, a.B, a.N, a.replay.capacity, a)
#define SWARM_TD_LAUNCH(NS, GS, NT)                                                       \
  do {                                                                                    \
    if (spec == SPEC_COMPLETE_GAT) SWARM_TD_LAUNCH1(NS, GS, NT, SPEC_COMPLETE_GAT);      \
    else if (spec == SPEC_COMPLETE_GCN) SWARM_TD_LAUNCH1(NS, GS, NT, SPEC_COMPLETE_GCN); \
    else SWARM_TD_LAUNCH1(NS, GS, NT, SPEC_RUNTIME);                                      \
  } while (0)
  if (a.N <= 8) SWARM_TD_LAUNCH(16, 8, 128 * 2);
  else if (a.N <= 16) SWARM_TD_LAUNCH(16, 16, 128 * 2);
  else SWARM_TD_LAUNCH(32, 32, 128);
#undef SWARM_TD_LAUNCH
#undef SWARM_TD_LAUNCH1
  return (int)hipGetLastError();
}

#if SWARM_STAMPS
int swarm_dbg_stamps_td(void* p) { return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_swarm_stamps), &p, sizeof(p)); }
#endif

int swarm_grad_reduce(const swarm_config* cfg, const swarm_adam_cfg* hp, const float* slabs, float* grad,
                      void* stream) {
  if (int e = check_td(cfg, hp)) return e;
  ReduceArgs a = {};
  a.n_slabs = td_blocks(cfg, hp->batch); a.slabs = slabs; a.grad = grad;
  hipLaunchKernelGGL(grad_reduce_kernel, dim3((N_PARAMS + 1 + kRedCols - 1) / kRedCols), dim3(kRedCols * kRedGroups), 0,
                     (hipStream_t)stream, a.slabs, a.ctrl, a.n_slabs, a.advance, a);
  return (int)hipGetLastError();
}

int swarm_reduce_advance(const swarm_config* cfg, const swarm_adam_cfg* hp, const float* slabs, const swarm_learner* lr,
                         int32_t replay_capacity, swarm_ctrl* ctrl, void* stream) {
  if (int e = check_td(cfg, hp)) return e;
  if (!lr || !ctrl || replay_capacity < 1) return SWARM_E_BADARG;
  ReduceArgs a = {};
  a.n_slabs = td_blocks(cfg, hp->batch); a.slabs = slabs; a.grad = lr->grad;
  a.advance = 1; a.lr = *lr; a.ctrl = ctrl;
  a.capacity = replay_capacity; a.B = cfg->n_envs; a.N = cfg->n_agents; a.batch = hp->batch;
  a.hp = *hp;
  a.k0 = (uint32_t)(cfg->seed & 0xFFFFFFFFu) ^ ((uint32_t)cfg->env_offset * 0x9E3779B9u);
  a.k1 = (uint32_t)(cfg->seed >> 32);
  hipLaunchKernelGGL(grad_reduce_kernel, dim3((N_PARAMS + 1 + kRedCols - 1) / kRedCols), dim3(kRedCols * kRedGroups), 0,
                     (hipStream_t)stream, a.slabs, a.ctrl, a.n_slabs, a.advance, a);
  return (int)hipGetLastError();
}

static int launch_adam(const swarm_config* cfg, const swarm_adam_cfg* hp, float* params, float* target, float* m,
                       float* v, const float* grad, int32_t cap, swarm_ctrl* ctrl, int flush, void* stream) {
  AdamArgs a = {};
  a.hp = *hp; a.B = cfg->n_envs; a.N = cfg->n_agents; a.capacity = cap; a.flush = flush;
  a.params = params; a.target = target; a.m = m; a.v = v; a.grad = grad; a.ctrl = ctrl;
  hipLaunchKernelGGL(adam_kernel, dim3(1), dim3(kAdamNT), 0, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

__global__ void sample_prepare_kernel(const swarm_ctrl* C, int capacity, int B, int batch, uint32_t k0, uint32_t k1,
                                      int32_t* out) {
  const uint32_t cap = (uint32_t)capacity;
  const uint32_t filled = C->filled_slots;
  const uint32_t vs = filled + 1 < cap ? filled + 1 : cap;
  const uint32_t ng = vs * (uint32_t)B;
  if (ng < (uint32_t)batch) return;
  const SampleKey sk = sample_key(ng, k0, k1, C->tick);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < batch; i += gridDim.x * blockDim.x)
    out[i] = (int32_t)sample_index((uint32_t)i, sk);
}

int swarm_sample_prepare(const swarm_config* cfg, const swarm_adam_cfg* hp, int32_t replay_capacity,
                         const swarm_ctrl* ctrl, int32_t* samples, void* stream) {
  if (int e = check_td(cfg, hp)) return e;
  if (!ctrl || !samples || replay_capacity < 1) return SWARM_E_BADARG;
  const uint32_t k0 = (uint32_t)(cfg->seed & 0xFFFFFFFFu) ^ ((uint32_t)cfg->env_offset * 0x9E3779B9u);
  hipLaunchKernelGGL(sample_prepare_kernel, dim3((hp->batch + 255) / 256), dim3(256), 0, (hipStream_t)stream, ctrl,
                     replay_capacity, cfg->n_envs, hp->batch, k0, (uint32_t)(cfg->seed >> 32), samples);
  return (int)hipGetLastError();
}

int swarm_adam_step(const swarm_config* cfg, const swarm_adam_cfg* hp, float* params, float* target, float* adam_m,
                    float* adam_v, const float* grad, int32_t replay_capacity, swarm_ctrl* ctrl, void* stream) {
  if (int e = check_td(cfg, hp)) return e;
  if (!params || !target || !adam_m || !adam_v || !grad || !ctrl || replay_capacity < 1) return SWARM_E_BADARG;
  return launch_adam(cfg, hp, params, target, adam_m, adam_v, grad, replay_capacity, ctrl, 0, stream);
}

int swarm_adam_flush(const swarm_config* cfg, const swarm_adam_cfg* hp, const swarm_learner* lr, swarm_ctrl* ctrl,
                     void* stream) {
  if (int e = check_td(cfg, hp)) return e;
  if (!lr || !ctrl) return SWARM_E_BADARG;
  return launch_adam(cfg, hp, lr->w_cur, lr->target, lr->m_cur, lr->v_cur, lr->grad, 1, ctrl, 1, stream);
}

int swarm_ctrl_init(const swarm_adam_cfg* hp, float eps, swarm_ctrl* ctrl, void* stream) {
  if (!hp || !ctrl) return SWARM_E_BADARG;
  hipLaunchKernelGGL(ctrl_init_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, *hp, eps, ctrl);
  return (int)hipGetLastError();
}

int swarm_ctrl_advance(const swarm_config* cfg, const swarm_replay* replay, swarm_ctrl* ctrl, void* stream) {
  if (!cfg || !ctrl) return SWARM_E_BADARG;
  hipLaunchKernelGGL(ctrl_advance_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, ctrl,
                     replay ? replay->capacity : 1);
  return (int)hipGetLastError();
}

}  // extern "C"
