// swarm_td.hip — learning side of the hot path: replay sample, TD loss, hand-written
// backward through GCN (PyG GATConv + MLP), deterministic gradient reduction,
// clip_grad_norm_ and Adam.  gfx950 only.
//
// Reference: DQNTrainer.train_step_dqn (src/training/train_gcn_dqn.py:112-137),
// GraphReplayBuffer.sample (:38-45), Adam(lr=1e-3) (:85), target sync (:131-133).
//
// One wave per tile of E = 32/N sampled graphs.  Backward per tile:
//   dQ[a] = (Q[a]-y) * 2/M                      (MSELoss mean, gather)
//   dR = W2[a]^T dQ ; dZ = dR * [Z>0] ; dT = W1^T dZ (MFMA) ; dOut = dT * (1 - t^2)
//   GAT: g_uv = dOut_v.h_u ; de_uv = c_uv (g_uv - sum_w c_wv g_wv) ; dp = de * leaky'(p)
//        da_dst[v] = sum_u dp_uv ; da_src[u] = sum_v dp_uv ; dh_u = sum_v c_uv dOut_v + da_src att_src + da_dst att_dst
//   parameter sums over the tile's nodes: dW1 = dZ^T T, dW2 = dQ^T R, dW = dh^T X on MFMA
//   (32x32x2 f32, node index as K), vectors by LDS column sums.
// Each block writes one slab [N_PARAMS + 1] (last = sum of squared TD errors);
// swarm_grad_reduce sums slabs in a fixed order (bitwise run-to-run reproducible).
#include <stdlib.h>

#include "swarm_adam.h"
#include "swarm_tile.h"

namespace swarm {

template <int NMAX>
struct TdTileLds {
  WaveLds L;                      // online forward scratch (H rows, scores, positions)
  WaveLds LT;                     // target forward scratch
  float T[kTile][kHsStride];      // tanh(conv out), natural order    } reused as this tile's
  float R[kTile][kHsStride];      // relu(lin1)                        } partial slab after the
  float dZ[kTile][kHsStride];     //                                   } parameter products
  float dO[kTile][kHsStride];     // dL/d conv out
  float dH[kTile][kHsStride];     // dL/d h
  float X[kTile][9];              // features (k < 8)
  float cm[kTile][NMAX + 1];      // c[target slot][source agent]
  float dp[kTile][NMAX + 1];      // dp[target slot][source agent]
  float y[kTile];                 // TD targets from the target wave
  float gq[kTile];
  float das[kTile], dad[kTile];
  float d2[kTile];
  int act[kTile];
};
static_assert(5 * kTile * kHsStride >= N_PARAMS + 1, "partial slab fits the image area");

// tiles per block; each tile has an online wave and a target wave (2 * TPB waves)
template <int NMAX> constexpr int td_tpb_max() { return NMAX <= 16 ? 3 : 2; }

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

__device__ inline void store_acc_row(float (*img)[kHsStride], int v, int h, const float val[16]) {
#pragma unroll
  for (int q = 0; q < 4; ++q)
    *reinterpret_cast<float4*>(&img[v][8 * q + 4 * h]) = make_float4(val[4 * q], val[4 * q + 1], val[4 * q + 2], val[4 * q + 3]);
}

// D[i][j] = sum_node A_img[node][i] * B_img[node][j] over the 32 node slots (MFMA, K = node)
__device__ inline f32x16 mfma_nodesum(const float (*Aimg)[kHsStride], const float (*Bimg)[kHsStride], int lane) {
  f32x16 acc = {};
  const int h = lane >> 5, c = lane & 31;
#pragma unroll
  for (int s = 0; s < 16; ++s) acc = mfma32(Aimg[2 * s + h][c], Bimg[2 * s + h][c], acc);
  return acc;
}

// Waves 0..TPB-1: online network of tile w (forward with activations kept, backward,
// dW / att gradients); waves TPB..2TPB-1: target network of tile w-TPB (forward on s',
// y = r + gamma max Q_tgt), then the dW1 / dW2 / bias products while the online wave
// runs the GAT backward.  Every wave passes the same __syncthreads() sequence.
template <int NMAX, int TPB>
__global__ __launch_bounds__(128 * TPB) void td_kernel(TdArgs A) {
  static_assert(TPB <= td_tpb_max<NMAX>(), "LDS budget");
  __shared__ TdTileLds<NMAX> TW[TPB];
  __shared__ __attribute__((aligned(16))) float Pon[N_PARAMS_PAD];
  __shared__ __attribute__((aligned(16))) float Ptg[N_PARAMS_PAD];
  const int wave = threadIdx.x >> 6;
  const int tl = wave % TPB;
  const bool online = wave < TPB;
  TdTileLds<NMAX>& T = TW[tl];
  WaveLds& L = online ? T.L : T.LT;
  const int N = A.N;
  const Geom g = make_geom(blockIdx.x * TPB + tl, N, A.S);
  const int lane = g.lane, h = g.h;
  float* gslab = A.slabs + (size_t)blockIdx.x * (N_PARAMS + 1);
  float* slab = &T.T[0][0];       // this tile's partial slab (after the products)
  SWARM_STAMP(0);

  // ---- weights: both images' loads issued first (one round trip)
  ParamStage<128 * TPB> pon, ptg;
  pon.load(A.params, threadIdx.x);
  ptg.load(A.target, threadIdx.x);
  // ---- skip while the replay holds fewer than `batch` graphs (train_gcn_dqn.py:113-115)
  const uint32_t filled = A.ctrl->filled_slots;
  const uint32_t cap = (uint32_t)A.replay.capacity;
  const uint32_t valid_slots = filled + 1 < cap ? filled + 1 : cap;
  const uint32_t n_graphs = valid_slots * (uint32_t)A.B;
  if (n_graphs < (uint32_t)A.S) {
    for (int p = threadIdx.x; p <= N_PARAMS; p += 128 * TPB) gslab[p] = 0.0f;
    return;
  }
  SWARM_STAMP(1);
  // ---- sample (GraphReplayBuffer.sample: random.sample -> keyed permutation)
  uint32_t gid = 0;
  if (A.sample_in) {
    gid = (uint32_t)A.sample_in[g.valid ? g.env : 0];
  } else {
    const SampleKey sk = sample_key(n_graphs, A.k0 ^ ((uint32_t)A.env_offset * 0x9E3779B9u), A.k1, A.ctrl->tick);
    gid = sample_index((uint32_t)(g.valid ? g.env : 0), sk);
  }
  if (A.sample_out && online && g.valid && h == 0 && g.agent == 0) A.sample_out[g.env] = (int32_t)gid;
  SWARM_STAMP(2);
  const uint32_t slot = gid / (uint32_t)A.B, genv = gid % (uint32_t)A.B;
  const size_t ri = ((size_t)slot * A.B + genv) * N + g.agent;
  const float4 st = reinterpret_cast<const float4*>(online ? A.replay.s : A.replay.s_next)[ri];
  const float rew = A.replay.r[ri];
  const int act = g.valid ? (int)A.replay.a[ri] : 0;
  pon.store(Pon, threadIdx.x);
  ptg.store(Ptg, threadIdx.x);

  FwdState F;
  F.x[0] = st.x; F.x[1] = st.y; F.x[2] = st.z; F.x[3] = st.w;
  F.x[4] = kGoalX; F.x[5] = kGoalY; F.x[6] = (float)g.agent; F.x[7] = 0.0f;
  if (!g.valid) {
#pragma unroll
    for (int k = 0; k < 8; ++k) F.x[k] = 0.0f;
  }
  if (h == 0) { L.px[g.v] = F.x[0]; L.py[g.v] = F.x[1]; }
  int mult[NMAX];
  float c[NMAX];
  __syncthreads();
  SWARM_STAMP(3);
  // ---- forwards: online on s (activations kept), target on s' (train_gcn_dqn.py:119-121)
  tile_forward<NMAX, 16>(online ? Pon : Ptg, g, N, A.graph, A.k, A.conv, nullptr, L, F, mult, c);
  if (!online) {
    float qmax = F.q[0];
#pragma unroll
    for (int a = 1; a < kActions; ++a) qmax = fmaxf(qmax, F.q[a]);
    if (h == 0) T.y[g.v] = rew + A.gamma * qmax;
  }
  SWARM_STAMP(4);
  __syncthreads();
  SWARM_STAMP(5);

  const float* P = Pon;
  float delta = 0.0f;
  float dO[16];
  if (online) {
    float qa = F.q[0];
#pragma unroll
    for (int a = 1; a < kActions; ++a) qa = (act == a) ? F.q[a] : qa;
    delta = g.valid ? (qa - T.y[g.v]) : 0.0f;
    const float gq = delta * A.grad_scale;
    if (!g.valid) {
#pragma unroll
      for (int u = 0; u < NMAX; ++u) c[u] = 0.0f;
    }
    // ---- MLP backward
    float dZ[16], dT[16];
    {
      float w2[16];
      load_vec_acc(P + OFF_W2 + act * kHidden, h, w2);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float dR = w2[r] * gq;
        dZ[r] = F.zr[r] > 0.0f ? dR : 0.0f;
      }
    }
    mfma_lin32_t(P + OFF_W1, g, dZ, dT);
#pragma unroll
    for (int r = 0; r < 16; ++r) dO[r] = dT[r] * (1.0f - F.t[r] * F.t[r]);
    SWARM_STAMP(6);
    store_acc_row(T.T, g.v, h, F.t);
    store_acc_row(T.R, g.v, h, F.zr);
    store_acc_row(T.dZ, g.v, h, dZ);
    store_acc_row(T.dO, g.v, h, dO);
    if (h == 0) {
#pragma unroll
      for (int k = 0; k < 8; ++k) T.X[g.v][k] = k < kFeat ? F.x[k] : 0.0f;
      T.X[g.v][8] = 0.0f;
      T.gq[g.v] = gq;
      T.act[g.v] = act;
      T.d2[g.v] = delta * delta;
#pragma unroll
      for (int u = 0; u < NMAX; ++u)
        if (u < N) T.cm[g.v][u] = c[u];
    }
  }
  __syncthreads();   // images of every tile ready
  SWARM_STAMP(7);

  const int col = lane & 31;
  // target-wave products (registers) while the online wave does the GAT backward
  f32x16 dW1 = {}, dW2 = {};
  float s_bias = 0.0f, s_b1 = 0.0f, s_b2 = 0.0f, s_loss = 0.0f;
  float da_s = 0.0f, da_d = 0.0f;
  if (!online) {
    dW1 = mfma_nodesum(T.dZ, T.T, lane);                       // dW1[i][hid]
#pragma unroll
    for (int s = 0; s < 16; ++s) {                             // dW2[a][hid]
      const int n = 2 * s + h;
      const float a = (T.act[n] == col) ? T.gq[n] : 0.0f;
      dW2 = mfma32(a, T.R[n][col], dW2);
    }
    if (h == 0) {
      for (int n = 0; n < kTile; ++n) s_bias = s_bias + T.dO[n][col];
    } else {
      for (int n = 0; n < kTile; ++n) s_b1 = s_b1 + T.dZ[n][col];
    }
    if (lane < kActions) {
      for (int n = 0; n < kTile; ++n) s_b2 = s_b2 + (T.act[n] == lane ? T.gq[n] : 0.0f);
    } else if (lane == 63) {
      for (int n = 0; n < kTile; ++n) s_loss = s_loss + T.d2[n];
    }
  } else if (A.conv == SWARM_CONV_GAT) {
    // ---- GAT backward (attention part), branch-free over the env's sources u
    float gu[NMAX];
#pragma unroll
    for (int u = 0; u < NMAX; ++u) {
      gu[u] = 0.0f;
      if (u < N) {
        const float* row = &L.hs[g.base + u][4 * h];
        float p = 0.0f;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 hv = *reinterpret_cast<const float4*>(row + 8 * q);
          p = p + dO[4 * q] * hv.x;
          p = p + dO[4 * q + 1] * hv.y;
          p = p + dO[4 * q + 2] * hv.z;
          p = p + dO[4 * q + 3] * hv.w;
        }
        gu[u] = p;
      }
    }
    float G = 0.0f;
#pragma unroll
    for (int u = 0; u < NMAX; ++u) {
      if (u < N) gu[u] = gu[u] + xor32(gu[u]);
      if (u < N) G = G + c[u] * gu[u];
    }
#pragma unroll
    for (int u = 0; u < NMAX; ++u) {
      float dpu = 0.0f;
      if (u < N) {
        const float de = c[u] * (gu[u] - G);
        const float pre = L.ssrc[g.base + u] + F.sdst;
        dpu = pre > 0.0f ? de : de * kLeakySlope;
      }
      da_d = da_d + dpu;
      if (u < N && h == 0) T.dp[g.v][u] = dpu;
    }
  }
  __syncthreads();   // dp ready
  SWARM_STAMP(8);
  if (online) {
    if (A.conv == SWARM_CONV_GAT) {
      float col_dp[NMAX];
#pragma unroll
      for (int w = 0; w < NMAX; ++w) col_dp[w] = T.dp[g.base + (w < N ? w : 0)][g.agent];
#pragma unroll
      for (int w = 0; w < NMAX; ++w)
        if (w < N) da_s = da_s + col_dp[w];
    }
    if (!g.valid) { da_s = 0.0f; da_d = 0.0f; }
    // ---- dh = messages + attention-coefficient terms
    float dh[16];
    float as[16], ad[16];
    load_vec_acc(P + OFF_ATT_SRC, h, as);
    load_vec_acc(P + OFF_ATT_DST, h, ad);
#pragma unroll
    for (int r = 0; r < 16; ++r) dh[r] = 0.0f;
#pragma unroll
    for (int w = 0; w < NMAX; ++w) {
      if (w < N) {
        const float cw = g.valid ? T.cm[g.base + w][g.agent] : 0.0f;   // c[target w][source me]
        const float* row = &T.dO[g.base + w][4 * h];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 dv = *reinterpret_cast<const float4*>(row + 8 * q);
          dh[4 * q] = dh[4 * q] + cw * dv.x;
          dh[4 * q + 1] = dh[4 * q + 1] + cw * dv.y;
          dh[4 * q + 2] = dh[4 * q + 2] + cw * dv.z;
          dh[4 * q + 3] = dh[4 * q + 3] + cw * dv.w;
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) dh[r] = (dh[r] + da_s * as[r]) + da_d * ad[r];
    store_acc_row(T.dH, g.v, h, dh);
    if (h == 0) { T.das[g.v] = da_s; T.dad[g.v] = da_d; }
  }
  __syncthreads();   // dH ready
  SWARM_STAMP(9);
  f32x16 dW = {};
  float s_as = 0.0f, s_ad = 0.0f;
  if (online) {
#pragma unroll
    for (int s = 0; s < 16; ++s) {                             // dW[hid][k]
      const int n = 2 * s + h;
      dW = mfma32(T.dH[n][col], col < 8 ? T.X[n][col] : 0.0f, dW);
    }
    if (h == 0) {
      for (int n = 0; n < kTile; ++n) s_as = s_as + T.das[n] * L.hs[n][col];
    } else {
      for (int n = 0; n < kTile; ++n) s_ad = s_ad + T.dad[n] * L.hs[n][col];
    }
  }
  SWARM_STAMP(10);
  __syncthreads();   // every image read done: the image area becomes the partial slab
  if (online) {
    if (col < kFeat) {
#pragma unroll
      for (int r = 0; r < 16; ++r) slab[OFF_W + acc_row(r, h) * kFeat + col] = dW[r];
    }
    if (h == 0) slab[OFF_ATT_SRC + col] = s_as;
    else        slab[OFF_ATT_DST + col] = s_ad;
  } else {
#pragma unroll
    for (int r = 0; r < 16; ++r) slab[OFF_W1 + acc_row(r, h) * kHidden + col] = dW1[r];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int a = acc_row(r, h);
      if (a < kActions) slab[OFF_W2 + a * kHidden + col] = dW2[r];
    }
    if (h == 0) slab[OFF_BIAS + col] = s_bias;
    else        slab[OFF_B1 + col] = s_b1;
    if (lane < kActions) slab[OFF_B2 + lane] = s_b2;
    else if (lane == 63) slab[N_PARAMS] = s_loss;
  }
  __syncthreads();
  SWARM_STAMP(11);
  // fixed-order sum of the block's TPB partial slabs -> one global slab
  for (int p = threadIdx.x; p <= N_PARAMS; p += 128 * TPB) {
    float acc = (&TW[0].T[0][0])[p];
#pragma unroll
    for (int w = 1; w < TPB; ++w) acc = acc + (&TW[w].T[0][0])[p];
    gslab[p] = acc;
  }
  SWARM_STAMP(12);
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
  float beta1, beta2;
  int32_t* sample_next;   // fused tick: replay indices of the NEXT tick's TD batch
  uint32_t k0, k1;        // sampling key (seed ^ rank salt)
};

// 1024 threads = 64 columns x 16 slab groups; group g sums a contiguous run of at most
// 16 slabs with every load issued before the ordered adds, then the 16 group sums are
// added in group order (fixed order -> bitwise reproducible run to run).
constexpr int kRedGroups = 16;
__global__ __launch_bounds__(64 * kRedGroups) void grad_reduce_kernel(ReduceArgs A) {
  __shared__ float part[kRedGroups][64];
  const int c = threadIdx.x & 63;
  const int col = blockIdx.x * 64 + c;
  const int q = threadIdx.x >> 6;
  const int per = (A.n_slabs + kRedGroups - 1) / kRedGroups;
  const int b0 = q * per, b1 = min(A.n_slabs, b0 + per);
  float s = 0.0f;
  if (col <= N_PARAMS) {
    for (int b = b0; b < b1; b += 16) {
      float v[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) v[j] = (b + j < b1) ? A.slabs[(size_t)(b + j) * (N_PARAMS + 1) + col] : 0.0f;
#pragma unroll
      for (int j = 0; j < 16; ++j) s = s + v[j];
    }
  }
  if (A.advance && col < N_PARAMS) {   // ping-pong copy-back, one array per group
    if (q == 0) A.lr.w_cur[col] = A.lr.w_nxt[col];
    else if (q == 1) A.lr.m_cur[col] = A.lr.m_nxt[col];
    else if (q == 2) A.lr.v_cur[col] = A.lr.v_nxt[col];
  }
  part[q][c] = s;
  // the block holding column N_PARAMS also owns the control block: it reads ctrl
  // before its single writer updates it, and draws the next tick's sample indices
  // (the permutation the TD kernel would otherwise compute on its critical path)
  const bool owner = A.advance && (blockIdx.x == (N_PARAMS / 64));
  uint32_t c_tick = 0, c_filled = 0;
  if (owner) { c_tick = A.ctrl->tick; c_filled = A.ctrl->filled_slots; }
  __syncthreads();
  if (owner && A.sample_next) {
    const uint32_t cap = (uint32_t)A.capacity;
    const uint32_t f1 = c_filled + 1 < cap ? c_filled + 1 : cap;           // filled after this tick
    const uint32_t vs = f1 + 1 < cap ? f1 + 1 : cap;                        // valid slots next tick
    const uint32_t ng = vs * (uint32_t)A.B;
    if (ng >= (uint32_t)A.batch) {
      const SampleKey sk = sample_key(ng, A.k0, A.k1, c_tick + 1);
      for (int i = threadIdx.x; i < A.batch; i += blockDim.x) A.sample_next[i] = (int32_t)sample_index((uint32_t)i, sk);
    }
  }
  if (q == 0 && col <= N_PARAMS) {
    float tot = part[0][c];
#pragma unroll
    for (int gi = 1; gi < kRedGroups; ++gi) tot = tot + part[gi][c];
    A.grad[col] = tot;
    if (A.advance && col == N_PARAMS) {   // one thread: record the pending update, advance the tick
      swarm_ctrl* C = A.ctrl;
      const uint32_t cap = (uint32_t)A.capacity;
      const uint32_t filled = C->filled_slots;
      const uint32_t valid_slots = filled + 1 < cap ? filled + 1 : cap;
      const uint32_t trained = valid_slots * (uint32_t)A.B >= (uint32_t)A.batch ? 1u : 0u;
      if (C->trained) {                                   // applied by this tick's act kernel
        C->adam_step = C->adam_step + 1;
        ctrl_set_double(C, CTRL_B1POW, ctrl_get_double(C, CTRL_B1POW) * (double)A.beta1);
        ctrl_set_double(C, CTRL_B2POW, ctrl_get_double(C, CTRL_B2POW) * (double)A.beta2);
      }
      C->trained = trained;
      C->loss = trained ? tot / (float)((size_t)A.batch * A.N) : 0.0f;
      C->tick = C->tick + 1;
      C->write_slot = (C->write_slot + 1) % cap;
      C->filled_slots = valid_slots;
    }
  }
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
  const double b1pow = ctrl_get_double(C, CTRL_B1POW) * (double)A.hp.beta1;
  const double b2pow = ctrl_get_double(C, CTRL_B2POW) * (double)A.hp.beta2;
  const bool train = A.flush ? (C->trained != 0u) : (valid_slots * (uint32_t)A.B >= (uint32_t)A.hp.batch);
  // target sync: unfused = after the TD step of tick `tick` ((tick+1) % every); flush = the
  // fused tick already advanced ctrl, so the pending update belongs to tick - 1
  const bool sync = ((A.flush ? tick : tick + 1) % (uint32_t)A.hp.update_target_every) == 0u;
  __syncthreads();   // every thread has read ctrl before thread 0 rewrites it
  float gn = 0.0f;
  if (train) {
    gn = adam_apply(R, A.hp, b1pow, b2pow, tid, red);
    store4(A.params, R.w, R.wt, tid);
    store4(A.m, R.m, R.mt, tid);
    store4(A.v, R.v, R.vt, tid);
    if (sync) store4(A.target, R.w, R.wt, tid);
  }
  if (tid == 0) {
    if (train) {
      C->adam_step = step;
      C->grad_norm = gn;
      ctrl_set_double(C, CTRL_B1POW, b1pow);
      ctrl_set_double(C, CTRL_B2POW, b2pow);
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

__global__ void ctrl_advance_kernel(swarm_ctrl* C, int capacity) {
  const uint32_t cap = (uint32_t)(capacity > 0 ? capacity : 1);
  C->tick = C->tick + 1;
  C->write_slot = (C->write_slot + 1) % cap;
  C->filled_slots = C->filled_slots + 1 < cap ? C->filled_slots + 1 : cap;
}

}  // namespace swarm

using namespace swarm;

namespace {
int td_tiles(const swarm_config* cfg, int batch) {
  const int E = kTile / cfg->n_agents;
  return (batch + E - 1) / E;
}
// tiles per TD block (each tile = online wave + target wave); SWARM_TD_TPB=1|2|3 overrides
int td_tpb_rt(int N) {
  static int env = [] { const char* e = getenv("SWARM_TD_TPB"); return e ? atoi(e) : 0; }();
  const int mx = N <= 16 ? 3 : 2;
  int t = (env >= 1 && env <= 3) ? env : 1;   // measured: 1 tile per block is fastest (256 blocks)
  return t < mx ? t : mx;
}
int td_blocks(const swarm_config* cfg, int batch) {
  const int w = td_tpb_rt(cfg->n_agents);
  return (td_tiles(cfg, batch) + w - 1) / w;
}
int td_max_blocks(const swarm_config* cfg, int batch) { return td_tiles(cfg, batch); }
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
  const int w = td_tpb_rt(a.N);
#define SW_TD(NM, W) hipLaunchKernelGGL((td_kernel<NM, W>), dim3(nb), dim3(128 * W), 0, st, a)
  if (a.N <= 8) { if (w == 1) SW_TD(8, 1); else if (w == 2) SW_TD(8, 2); else SW_TD(8, 3); }
  else if (a.N <= 16) { if (w == 1) SW_TD(16, 1); else if (w == 2) SW_TD(16, 2); else SW_TD(16, 3); }
  else { if (w == 1) SW_TD(32, 1); else SW_TD(32, 2); }
#undef SW_TD
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
  hipLaunchKernelGGL(grad_reduce_kernel, dim3((N_PARAMS + 1 + 63) / 64), dim3(64 * kRedGroups), 0, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

int swarm_reduce_advance(const swarm_config* cfg, const swarm_adam_cfg* hp, const float* slabs, const swarm_learner* lr,
                         int32_t replay_capacity, swarm_ctrl* ctrl, int32_t* sample_next, void* stream) {
  if (int e = check_td(cfg, hp)) return e;
  if (!lr || !ctrl || replay_capacity < 1) return SWARM_E_BADARG;
  ReduceArgs a = {};
  a.n_slabs = td_blocks(cfg, hp->batch); a.slabs = slabs; a.grad = lr->grad;
  a.advance = 1; a.lr = *lr; a.ctrl = ctrl;
  a.capacity = replay_capacity; a.B = cfg->n_envs; a.N = cfg->n_agents; a.batch = hp->batch;
  a.beta1 = hp->beta1; a.beta2 = hp->beta2;
  a.sample_next = sample_next;
  a.k0 = (uint32_t)(cfg->seed & 0xFFFFFFFFu) ^ ((uint32_t)cfg->env_offset * 0x9E3779B9u);
  a.k1 = (uint32_t)(cfg->seed >> 32);
  hipLaunchKernelGGL(grad_reduce_kernel, dim3((N_PARAMS + 1 + 63) / 64), dim3(64 * kRedGroups), 0, (hipStream_t)stream, a);
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

int swarm_ctrl_advance(const swarm_config* cfg, const swarm_replay* replay, swarm_ctrl* ctrl, void* stream) {
  if (!cfg || !ctrl) return SWARM_E_BADARG;
  hipLaunchKernelGGL(ctrl_advance_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, ctrl,
                     replay ? replay->capacity : 1);
  return (int)hipGetLastError();
}

}  // extern "C"
