// swarm_adam.h — clip_grad_norm_(max_norm) + Adam for the 1,673 GCN parameters,
// executed by one workgroup of NT threads with everything in registers.  The same
// code (same NT) runs in the fused act prologue (every block, redundantly, result
// into its LDS weight image), in swarm_adam_flush and in the unfused
// swarm_adam_step, so the three paths are bit-identical.
//
// Reference: train_gcn_dqn.py:125-126 (clip_grad_norm_(model.parameters(), 1);
// Adam(lr=1e-3)).  torch semantics restated: total = norm of the per-tensor L2 norms
// (computed here as the global L2 norm, equal up to rounding), coef = max_norm /
// (total + 1e-6) clamped to 1, grads *= coef; Adam
// single_tensor: m.lerp_(g, 1-b1); v = v*b2 + (1-b2) g g; denom = sqrt(v)/sqrt(bc2) + eps;
// w += -(lr/bc1) * m/denom.  bc = 1 - beta^step with beta^step kept as a running
// double product in the control block (python's beta ** step up to ~1e-16 relative).
#pragma once
#include "swarm_common.h"

namespace swarm {

constexpr int kAdamNT = 256;                           // threads of every Adam workgroup
constexpr int kAdamNF4 = N_PARAMS / 4;                 // 418 float4 = floats 0..1671
constexpr int kAdamNJ = (kAdamNF4 + kAdamNT - 1) / kAdamNT;
static_assert(kAdamNF4 * 4 + 1 == N_PARAMS, "one tail element (lin2.bias[8])");

// beta^step running products live in the control block (two doubles, words 10-13)
__device__ inline double ctrl_get_double(const swarm_ctrl* c, int word) {
  const uint32_t* p = &c->beta_pow[word];
  return __hiloint2double((int)p[1], (int)p[0]);
}
__device__ inline void ctrl_set_double(swarm_ctrl* c, int word, double v) {
  c->beta_pow[word] = (uint32_t)__double2loint(v);
  c->beta_pow[word + 1] = (uint32_t)__double2hiint(v);
}
constexpr int CTRL_B1POW = 0;   // beta_pow[0..1] = beta1^adam_step
constexpr int CTRL_B2POW = 2;   // beta_pow[2..3] = beta2^adam_step

// the hyper-parameters in double as torch.optim.Adam holds them (swarm_adam_cfg *_d; 0 = the
// float field): torch forms 1 - beta1 = 0.1, 1 - beta2 = 0.001 and the bias corrections from
// Python floats, and (float)(1 - (double)0.999f) is 1.3e-5 away from 0.001f, a systematic
// 200-ulp bias on v
__device__ inline double adam_lr(const swarm_adam_cfg& hp) { return hp.lr_d != 0.0 ? hp.lr_d : (double)hp.lr; }
__device__ inline double adam_beta1(const swarm_adam_cfg& hp) { return hp.beta1_d != 0.0 ? hp.beta1_d : (double)hp.beta1; }
__device__ inline double adam_beta2(const swarm_adam_cfg& hp) { return hp.beta2_d != 0.0 ? hp.beta2_d : (double)hp.beta2; }

// Adam scalars of the step after the one ctrl's beta powers describe (torch single_tensor:
// step_size = lr / bias_correction1, bias_correction2_sqrt = sqrt(bias_correction2), both
// in double), stored in ctrl as floats by whoever advances the powers, so the optimizer
// step itself carries no double-precision work.  One function for every path.
// b1pow / b2pow: beta^s after s steps -> the scalars of step s + 1
__device__ inline void adam_next_scalars(const swarm_adam_cfg& hp, double b1pow, double b2pow, float& step_size,
                                         float& inv_bc2) {
  const double b1n = b1pow * adam_beta1(hp);
  const double b2n = b2pow * adam_beta2(hp);
  step_size = (float)(adam_lr(hp) / (1.0 - b1n));
  inv_bc2 = 1.0f / (float)sqrt(1.0 - b2n);
}
__device__ inline void ctrl_store_next_scalars(swarm_ctrl* c, const swarm_adam_cfg& hp) {
  adam_next_scalars(hp, ctrl_get_double(c, CTRL_B1POW), ctrl_get_double(c, CTRL_B2POW), c->adam_step_size,
                    c->adam_inv_bc2);
}

struct AdamRegs {
  float4 g[kAdamNJ], w[kAdamNJ], m[kAdamNJ], v[kAdamNJ];
  float gt, wt, mt, vt;    // tail element N_PARAMS - 1

  // every load issued unconditionally (clamped index): one memory round trip
  __device__ inline void load(const float* __restrict__ grad, const float* __restrict__ w_, const float* __restrict__ m_,
                              const float* __restrict__ v_, int tid) {
#pragma unroll
    for (int j = 0; j < kAdamNJ; ++j) {
      const int i = min(tid + kAdamNT * j, kAdamNF4 - 1);
      g[j] = reinterpret_cast<const float4*>(grad)[i];
      w[j] = reinterpret_cast<const float4*>(w_)[i];
      m[j] = reinterpret_cast<const float4*>(m_)[i];
      v[j] = reinterpret_cast<const float4*>(v_)[i];
    }
    // the tail element as VECTOR loads (pointers moved into VGPRs): as scalar loads they were
    // issued only after the wave's first scalar wait and arrived one round trip late
    typedef const __attribute__((address_space(1))) float gfloat;   // global, not flat
    gfloat* tg = (gfloat*)(grad + (N_PARAMS - 1));
    gfloat* tw = (gfloat*)(w_ + (N_PARAMS - 1));
    gfloat* tm = (gfloat*)(m_ + (N_PARAMS - 1));
    gfloat* tv = (gfloat*)(v_ + (N_PARAMS - 1));
    asm volatile("" : "+v"(tg), "+v"(tw), "+v"(tm), "+v"(tv));
    gt = *tg; wt = *tw; mt = *tm; vt = *tv;
  }
};

template <int CTRL>
__device__ inline float adam_dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
// wave-wide sum, fixed order: DPP butterflies inside each 16-lane row (quad_perm xor-1,
// xor-2, row_half_mirror, row_mirror), then the four row sums in row order
__device__ inline float wave_sum(float x) {
  x = x + adam_dpp<0xB1>(x);
  x = x + adam_dpp<0x4E>(x);
  x = x + adam_dpp<0x141>(x);
  x = x + adam_dpp<0x140>(x);
  const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 0));
  const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 16));
  const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 32));
  const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 48));
  return ((r0 + r1) + r2) + r3;
}

// torch divides twice per element; here both divisions are reciprocal multiplies and
// the square root is v_sqrt_f32 (<= 1-2 ulp per step, inside the 2e-6 parameter
// tolerance of the parity tests).
__device__ inline void adam_elem(float g, float& w, float& m, float& v, float one_m_b1, float beta2,
                                 float one_m_b2, float inv_bc2_sqrt, float eps, float step_size) {
  m = m + one_m_b1 * (g - m);
  v = v * beta2;
  v = v + one_m_b2 * g * g;
  const float denom = __builtin_amdgcn_sqrtf(v) * inv_bc2_sqrt + eps;
  w = w + (-step_size) * (m * __builtin_amdgcn_rcpf(denom));
}

// One optimizer step in registers by the whole workgroup (kAdamNT threads; contains
// __syncthreads).  step_size / inv_bc2_sqrt: ctrl's scalars of this step.  Returns the
// pre-clip global norm.  red: LDS scratch of >= kAdamNT/64 floats.
template <int SB = -1>   // SB: diagnostic stamp base (SWARM_STAMPS builds only)
// one_m_b1 / one_m_b2: ctrl's (float)(1 - beta) (swarm_ctrl_init, from the double betas): read
// with the control block the prologue loads anyway, not from a kernarg double on its chain
__device__ inline float adam_apply(AdamRegs& R, const swarm_adam_cfg& hp, float step_size, float inv_bc2_sqrt,
                                   float one_m_b1, float one_m_b2, int tid, float* red) {
#define AD_STAMP(i) do { if (SB >= 0) SWARM_STAMP(SB + (i)); } while (0)
  const float inv_w = 1.0f / (float)hp.world_size;
  // clip_grad_norm_: the norm of the per-tensor norms == the global L2 norm up to rounding
  // (<= ~1e-7 relative on the clip coefficient); one fixed-order reduction
  float ss = 0.0f;
#pragma unroll
  for (int j = 0; j < kAdamNJ; ++j) {
    const int i = tid + kAdamNT * j;
    float4 g = R.g[j];
    if (hp.world_size > 1) { g.x = g.x * inv_w; g.y = g.y * inv_w; g.z = g.z * inv_w; g.w = g.w * inv_w; }
    R.g[j] = g;
    const float d = ((g.x * g.x + g.y * g.y) + g.z * g.z) + g.w * g.w;
    ss = ss + (i < kAdamNF4 ? d : 0.0f);
  }
  if (hp.world_size > 1) R.gt = R.gt * inv_w;
  if (tid == 0) ss = ss + R.gt * R.gt;
  AD_STAMP(0);
  constexpr int NW = kAdamNT / 64;
  {
    const float s = wave_sum(ss);
    if ((tid & 63) == 0) red[tid >> 6] = s;
  }
  __syncthreads();
  float nn = red[0];
#pragma unroll
  for (int w = 1; w < NW; ++w) nn = nn + red[w];
  // v_sqrt_f32 and a reciprocal multiply (<= 1 ulp each) instead of the correctly rounded
  // expansions: the clip coefficient is a serial chain every prologue waits on (0.075 us per
  // tick at C2, profiles/r02_ab_wpe.jsonl)
  const float total_norm = __builtin_amdgcn_sqrtf(nn);
  AD_STAMP(1);
  const float coef = hp.max_norm * __builtin_amdgcn_rcpf(total_norm + 1e-6f);
  const float clamped = coef < 1.0f ? coef : 1.0f;
  const float bc2_sqrt = inv_bc2_sqrt;   // reciprocal of sqrt(bias_correction2)
#pragma unroll
  for (int j = 0; j < kAdamNJ; ++j) {
    float4 g = R.g[j], w = R.w[j], m = R.m[j], v = R.v[j];
    adam_elem(g.x * clamped, w.x, m.x, v.x, one_m_b1, hp.beta2, one_m_b2, bc2_sqrt, hp.eps, step_size);
    adam_elem(g.y * clamped, w.y, m.y, v.y, one_m_b1, hp.beta2, one_m_b2, bc2_sqrt, hp.eps, step_size);
    adam_elem(g.z * clamped, w.z, m.z, v.z, one_m_b1, hp.beta2, one_m_b2, bc2_sqrt, hp.eps, step_size);
    adam_elem(g.w * clamped, w.w, m.w, v.w, one_m_b1, hp.beta2, one_m_b2, bc2_sqrt, hp.eps, step_size);
    R.w[j] = w; R.m[j] = m; R.v[j] = v;
  }
  adam_elem(R.gt * clamped, R.wt, R.mt, R.vt, one_m_b1, hp.beta2, one_m_b2, bc2_sqrt, hp.eps, step_size);
  AD_STAMP(2);
#undef AD_STAMP
  return total_norm;
}

__device__ inline void store4(float* __restrict__ dst, const float4* src, float tail, int tid) {
#pragma unroll
  for (int j = 0; j < kAdamNJ; ++j) {
    const int i = tid + kAdamNT * j;
    if (i < kAdamNF4) reinterpret_cast<float4*>(dst)[i] = src[j];
  }
  if (tid == 0) dst[N_PARAMS - 1] = tail;
}

// padded LDS weight image (lds_index, N_LDS_PARAMS floats)
__device__ inline void store_w_lds(float* __restrict__ lds, const AdamRegs& R, int tid) {
#pragma unroll
  for (int j = 0; j < kAdamNJ; ++j) {
    const int i = tid + kAdamNT * j;
    if (i < kAdamNF4) *reinterpret_cast<float4*>(lds + lds_index(4 * i)) = R.w[j];
  }
  if (tid == 0) lds[lds_index(N_PARAMS - 1)] = R.wt;
}

}  // namespace swarm
