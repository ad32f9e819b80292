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
#include "swarm_tile.h"

namespace swarm {

struct TdLds {
  WaveLds L;
  float T[kTile][kHsStride];      // tanh(conv out), natural order
  float R[kTile][kHsStride];      // relu(lin1)
  float dZ[kTile][kHsStride];
  float dO[kTile][kHsStride];     // dL/d conv out
  float dH[kTile][kHsStride];     // dL/d h
  float X[kTile][kHsStride];      // features, cols >= 7 zero
  float cm[kTile][kTile + 1];     // c[target slot][source agent]
  float dp[kTile][kTile + 1];     // dp[target slot][source agent]
  float gq[kTile];
  float das[kTile], dad[kTile];
  float d2[kTile];
  int act[kTile];
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

template <int NMAX>
__global__ __launch_bounds__(64) void td_kernel(TdArgs A) {
  __shared__ TdLds T;
  WaveLds& L = T.L;
  const int N = A.N;
  const Geom g = make_geom(blockIdx.x, N, A.S);
  const int lane = g.lane, h = g.h;
  float* slab = A.slabs + (size_t)blockIdx.x * (N_PARAMS + 1);

  // ---- skip while the replay holds fewer than `batch` graphs (train_gcn_dqn.py:113-115)
  const uint32_t filled = A.ctrl->filled_slots;
  const uint32_t cap = (uint32_t)A.replay.capacity;
  const uint32_t valid_slots = filled + 1 < cap ? filled + 1 : cap;
  const uint32_t n_graphs = valid_slots * (uint32_t)A.B;
  if (n_graphs < (uint32_t)A.S) {
    for (int p = lane; p <= N_PARAMS; p += 64) slab[p] = 0.0f;
    return;
  }

  // ---- sample (GraphReplayBuffer.sample: random.sample -> keyed permutation)
  uint32_t gid = 0;
  if (g.valid) {
    if (A.sample_in) gid = (uint32_t)A.sample_in[g.env];
    else gid = sample_index((uint32_t)g.env, n_graphs, A.k0 ^ ((uint32_t)A.env_offset * 0x9E3779B9u), A.k1,
                            A.ctrl->tick);
    if (A.sample_out && h == 0 && g.agent == 0) A.sample_out[g.env] = (int32_t)gid;
  }
  const uint32_t slot = gid / (uint32_t)A.B, genv = gid % (uint32_t)A.B;
  const size_t ri = ((size_t)slot * A.B + genv) * N + g.agent;
  float4 s0 = make_float4(0.f, 0.f, 0.f, 0.f), s1 = s0;
  float rew = 0.0f;
  int act = 0;
  if (g.valid) {
    s0 = reinterpret_cast<const float4*>(A.replay.s)[ri];
    s1 = reinterpret_cast<const float4*>(A.replay.s_next)[ri];
    rew = A.replay.r[ri];
    act = A.replay.a[ri];
  }

  FwdState F;
  int mult[NMAX];
  float c[NMAX];
  auto features = [&](const float4& s) {
    F.x[0] = s.x; F.x[1] = s.y; F.x[2] = s.z; F.x[3] = s.w;
    F.x[4] = kGoalX; F.x[5] = kGoalY; F.x[6] = (float)g.agent; F.x[7] = 0.0f;
    if (!g.valid) {
#pragma unroll
      for (int k = 0; k < 8; ++k) F.x[k] = 0.0f;
    }
    if (h == 0) { L.px[g.v] = F.x[0]; L.py[g.v] = F.x[1]; }
  };

  // ---- target network on s' (train_gcn_dqn.py:120-121)
  features(s1);
  __syncthreads();
  tile_forward<NMAX>(A.target, g, N, A.graph, A.k, A.conv, nullptr, L, F, mult, c);
  float qmax = F.q[0];
#pragma unroll
  for (int a = 1; a < kActions; ++a) qmax = fmaxf(qmax, F.q[a]);
  const float y = rew + A.gamma * qmax;
  __syncthreads();

  // ---- online network on s (keeps activations)
  features(s0);
  __syncthreads();
  tile_forward<NMAX>(A.params, g, N, A.graph, A.k, A.conv, nullptr, L, F, mult, c);
  float qa = F.q[0];
#pragma unroll
  for (int a = 1; a < kActions; ++a) qa = (act == a) ? F.q[a] : qa;
  const float delta = g.valid ? (qa - y) : 0.0f;
  const float gq = delta * A.grad_scale;
  if (!g.valid) {
#pragma unroll
    for (int u = 0; u < NMAX; ++u) c[u] = 0.0f;
  }

  const float* __restrict__ P = A.params;
  // ---- MLP backward
  float dZ[16], dT[16], dO[16];
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

  store_acc_row(T.T, g.v, h, F.t);
  store_acc_row(T.R, g.v, h, F.zr);
  store_acc_row(T.dZ, g.v, h, dZ);
  store_acc_row(T.dO, g.v, h, dO);
  if (h == 0) {
#pragma unroll
    for (int k = 0; k < 8; ++k) T.X[g.v][k] = k < kFeat ? F.x[k] : 0.0f;
    T.gq[g.v] = gq;
    T.act[g.v] = act;
    T.d2[g.v] = delta * delta;
#pragma unroll
    for (int u = 0; u < NMAX; ++u)
      if (u < N) T.cm[g.v][u] = c[u];
  } else {
#pragma unroll
    for (int k = 8; k < kTile; ++k) T.X[g.v][k] = 0.0f;
  }
  __syncthreads();

  // ---- GAT backward (attention part)
  float da_s = 0.0f, da_d = 0.0f;
  if (A.conv == SWARM_CONV_GAT) {
    float gu[NMAX];
    float G = 0.0f;
#pragma unroll
    for (int u = 0; u < NMAX; ++u) {
      gu[u] = 0.0f;
      if (u < N && c[u] != 0.0f) {
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
#pragma unroll
    for (int u = 0; u < NMAX; ++u) {
      if (u < N) gu[u] = gu[u] + xor32(gu[u]);
      if (u < N && c[u] != 0.0f) G = G + c[u] * gu[u];
    }
#pragma unroll
    for (int u = 0; u < NMAX; ++u) {
      float dpu = 0.0f;
      if (u < N && c[u] != 0.0f) {
        const float de = c[u] * (gu[u] - G);
        const float pre = L.ssrc[g.base + u] + F.sdst;
        dpu = pre > 0.0f ? de : de * kLeakySlope;
      }
      da_d = da_d + dpu;
      if (u < N && h == 0) T.dp[g.v][u] = dpu;
    }
    __syncthreads();
    for (int w = 0; w < N; ++w) da_s = da_s + T.dp[g.base + w][g.agent];
    if (!g.valid) { da_s = 0.0f; da_d = 0.0f; }
  }
  // ---- dh = messages + attention-coefficient terms
  float dh[16];
  {
    float as[16], ad[16];
    load_vec_acc(P + OFF_ATT_SRC, h, as);
    load_vec_acc(P + OFF_ATT_DST, h, ad);
#pragma unroll
    for (int r = 0; r < 16; ++r) dh[r] = 0.0f;
    for (int w = 0; w < N; ++w) {
      const float cw = g.valid ? T.cm[g.base + w][g.agent] : 0.0f;   // c[target w][source me]
      if (cw != 0.0f) {
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
  }
  store_acc_row(T.dH, g.v, h, dh);
  if (h == 0) { T.das[g.v] = da_s; T.dad[g.v] = da_d; }
  __syncthreads();

  // ---- parameter gradients summed over the tile's node slots
  const int col = lane & 31;
  {
    const f32x16 d = mfma_nodesum(T.dZ, T.T, lane);            // dW1[i][hid]
#pragma unroll
    for (int r = 0; r < 16; ++r) slab[OFF_W1 + acc_row(r, h) * kHidden + col] = d[r];
  }
  {
    f32x16 acc = {};                                             // dW2[a][hid]
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int n = 2 * s + h;
      const float a = (T.act[n] == col) ? T.gq[n] : 0.0f;
      acc = mfma32(a, T.R[n][col], acc);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int a = acc_row(r, h);
      if (a < kActions) slab[OFF_W2 + a * kHidden + col] = acc[r];
    }
  }
  {
    const f32x16 d = mfma_nodesum(T.dH, T.X, lane);            // dW[hid][k]
    if (col < kFeat) {
#pragma unroll
      for (int r = 0; r < 16; ++r) slab[OFF_W + acc_row(r, h) * kFeat + col] = d[r];
    }
  }
  {
    float s1v = 0.0f, s2v = 0.0f;
    if (h == 0) {
      for (int n = 0; n < kTile; ++n) { s1v = s1v + T.dO[n][col]; s2v = s2v + T.das[n] * L.hs[n][col]; }
      slab[OFF_BIAS + col] = s1v;
      slab[OFF_ATT_SRC + col] = s2v;
    } else {
      for (int n = 0; n < kTile; ++n) { s1v = s1v + T.dZ[n][col]; s2v = s2v + T.dad[n] * L.hs[n][col]; }
      slab[OFF_B1 + col] = s1v;
      slab[OFF_ATT_DST + col] = s2v;
    }
  }
  if (lane < kActions) {
    float s = 0.0f;
    for (int n = 0; n < kTile; ++n) s = s + (T.act[n] == lane ? T.gq[n] : 0.0f);
    slab[OFF_B2 + lane] = s;
  } else if (lane == 63) {
    float s = 0.0f;
    for (int n = 0; n < kTile; ++n) s = s + T.d2[n];
    slab[N_PARAMS] = s;
  }
}

// ---------------------------------------------------------------- slab reduction
// block = 256 threads covers 64 columns; thread (col, part) sums a contiguous quarter
// of the slabs, quarters combined in order: fixed order -> bitwise reproducible.
__global__ __launch_bounds__(256) void grad_reduce_kernel(int n_slabs, const float* __restrict__ slabs,
                                                          float* __restrict__ grad) {
  __shared__ float part[4][64];
  const int col = blockIdx.x * 64 + (threadIdx.x & 63);
  const int q = threadIdx.x >> 6;
  const int per = (n_slabs + 3) / 4;
  const int b0 = q * per, b1 = min(n_slabs, b0 + per);
  float s = 0.0f;
  if (col <= N_PARAMS)
    for (int b = b0; b < b1; ++b) s = s + slabs[(size_t)b * (N_PARAMS + 1) + col];
  part[q][threadIdx.x & 63] = s;
  __syncthreads();
  if (q == 0 && col <= N_PARAMS) {
    const int c = threadIdx.x & 63;
    grad[col] = ((part[0][c] + part[1][c]) + part[2][c]) + part[3][c];
  }
}

// ---------------------------------------------------------------- clip + Adam + target sync
struct AdamArgs {
  float lr, beta1, beta2, eps, max_norm;
  int batch, update_every, world, B, N;
  float* params;
  float* target;
  float* m;
  float* v;
  const float* grad;
  swarm_ctrl* ctrl;
  int capacity;
};

__device__ inline float block_sum_1024(float x, float* sh) {
  const int t = threadIdx.x;
  for (int o = 32; o > 0; o >>= 1) x = x + __shfl_xor(x, o, 64);
  __syncthreads();
  if ((t & 63) == 0) sh[t >> 6] = x;
  __syncthreads();
  float s = 0.0f;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s = s + sh[w];
  return s;
}

__global__ __launch_bounds__(1024) void adam_kernel(AdamArgs A) {
  __shared__ float sh[16];
  __shared__ float tnorm[8];
  const int t = threadIdx.x;
  swarm_ctrl* C = A.ctrl;
  const uint32_t filled = C->filled_slots;
  const uint32_t cap = (uint32_t)A.capacity;
  const uint32_t valid_slots = filled + 1 < cap ? filled + 1 : cap;
  const bool train = valid_slots * (uint32_t)A.B >= (uint32_t)A.batch;
  const uint32_t tick = C->tick;
  const uint32_t step = C->adam_step;
  __syncthreads();
  if (train) {
    const float inv_w = 1.0f / (float)A.world;
    // per-tensor L2 norms, then the norm of norms (torch clip_grad_norm_)
    const int offs[9] = {OFF_ATT_SRC, OFF_ATT_DST, OFF_BIAS, OFF_W, OFF_W1, OFF_B1, OFF_W2, OFF_B2, N_PARAMS};
    for (int ti = 0; ti < 8; ++ti) {
      float ss = 0.0f;
      for (int p = offs[ti] + t; p < offs[ti + 1]; p += blockDim.x) {
        const float gg = A.world > 1 ? A.grad[p] * inv_w : A.grad[p];
        ss = ss + gg * gg;
      }
      const float tot = block_sum_1024(ss, sh);
      if (t == 0) tnorm[ti] = sqrtf(tot);
      __syncthreads();
    }
    float nn = 0.0f;
    for (int ti = 0; ti < 8; ++ti) nn = nn + tnorm[ti] * tnorm[ti];
    const float total_norm = sqrtf(nn);
    const float coef = A.max_norm / (total_norm + 1e-6f);
    const float clamped = coef < 1.0f ? coef : 1.0f;
    const double stepd = (double)(step + 1);
    const double bc1 = 1.0 - pow((double)A.beta1, stepd);
    const double bc2 = 1.0 - pow((double)A.beta2, stepd);
    const float step_size = (float)((double)A.lr / bc1);
    const float bc2_sqrt = (float)sqrt(bc2);
    const float one_m_b1 = (float)(1.0 - (double)A.beta1);
    const float one_m_b2 = (float)(1.0 - (double)A.beta2);
    const bool sync = ((tick + 1) % (uint32_t)A.update_every) == 0u;
    for (int p = t; p < N_PARAMS; p += blockDim.x) {
      float gg = A.world > 1 ? A.grad[p] * inv_w : A.grad[p];
      gg = gg * clamped;
      float m = A.m[p], v = A.v[p];
      m = m + one_m_b1 * (gg - m);                       // exp_avg.lerp_(grad, 1-beta1)
      v = v * A.beta2;
      v = v + one_m_b2 * gg * gg;                        // addcmul_(grad, grad, 1-beta2)
      const float denom = sqrtf(v) / bc2_sqrt + A.eps;
      const float np = A.params[p] + (-step_size) * (m / denom);
      A.m[p] = m; A.v[p] = v; A.params[p] = np;
      if (sync) A.target[p] = np;
    }
    if (t == 0) {
      C->adam_step = step + 1;
      C->loss = A.grad[N_PARAMS] / (float)((size_t)A.batch * A.N) / (float)A.world;
      C->grad_norm = total_norm;
      C->trained = 1u;
    }
  } else if (t == 0) {
    C->loss = 0.0f;
    C->grad_norm = 0.0f;
    C->trained = 0u;
  }
  if (t == 0) {
    C->tick = tick + 1;
    C->write_slot = (C->write_slot + 1) % cap;
    C->filled_slots = filled + 1 < cap ? filled + 1 : cap;
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
int td_blocks(const swarm_config* cfg, int batch) {
  const int E = kTile / cfg->n_agents;
  return (batch + E - 1) / E;
}
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
  return (int64_t)td_blocks(cfg, batch) * (N_PARAMS + 1);
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
  if (a.N <= 8) hipLaunchKernelGGL((td_kernel<8>), dim3(nb), dim3(64), 0, st, a);
  else if (a.N <= 16) hipLaunchKernelGGL((td_kernel<16>), dim3(nb), dim3(64), 0, st, a);
  else hipLaunchKernelGGL((td_kernel<32>), dim3(nb), dim3(64), 0, st, a);
  return (int)hipGetLastError();
}

int swarm_grad_reduce(const swarm_config* cfg, const swarm_adam_cfg* hp, const float* slabs, float* grad,
                      void* stream) {
  if (int e = check_td(cfg, hp)) return e;
  const int nb = td_blocks(cfg, hp->batch);
  hipLaunchKernelGGL(grad_reduce_kernel, dim3((N_PARAMS + 1 + 63) / 64), dim3(256), 0, (hipStream_t)stream, nb,
                     slabs, grad);
  return (int)hipGetLastError();
}

int swarm_adam_step(const swarm_config* cfg, const swarm_adam_cfg* hp, float* params, float* target, float* adam_m,
                    float* adam_v, const float* grad, int32_t replay_capacity, swarm_ctrl* ctrl, void* stream) {
  if (int e = check_td(cfg, hp)) return e;
  if (!params || !target || !adam_m || !adam_v || !grad || !ctrl || replay_capacity < 1) return SWARM_E_BADARG;
  AdamArgs a = {};
  a.lr = hp->lr; a.beta1 = hp->beta1; a.beta2 = hp->beta2; a.eps = hp->eps; a.max_norm = hp->max_norm;
  a.batch = hp->batch; a.update_every = hp->update_target_every; a.world = hp->world_size;
  a.B = cfg->n_envs; a.N = cfg->n_agents;
  a.params = params; a.target = target; a.m = adam_m; a.v = adam_v; a.grad = grad; a.ctrl = ctrl;
  a.capacity = replay_capacity;
  hipLaunchKernelGGL(adam_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

int swarm_ctrl_advance(const swarm_config* cfg, const swarm_replay* replay, swarm_ctrl* ctrl, void* stream) {
  if (!cfg || !ctrl) return SWARM_E_BADARG;
  hipLaunchKernelGGL(ctrl_advance_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, ctrl,
                     replay ? replay->capacity : 1);
  return (int)hipGetLastError();
}

}  // extern "C"
