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
//
// The squared global norm has ONE fixed summation order on every path (ABI 10, swarm_hip.h
// SWARM_GRAD_SQ_BASE): per float4 i of parameters 4i..4i+3, d[i] = ((g0^2 + g1^2) + g2^2) + g3^2
// (the tail parameter 1672 alone in d[418]); per group j of four float4s (16 parameters),
// sq[j] = (d[4j] + d[4j+1]) + (d[4j+2] + d[4j+3]); then wave_sum over lanes l = 0..63 of
// sq[l] + sq[l + 64].  The slab reduce forms sq[j] for its 16 columns as it writes them, so the
// fused tick's prologue (SWARM_ADAM_F_NORM_PARTIALS) loads 105 partials with its other operands
// and every wave forms the norm alone, with no block barrier in front of the Adam elements;
// without the flag (and in swarm_adam_step / _flush) the block forms the same sums from grad.
#pragma once
#include "swarm_common.h"

namespace swarm {

constexpr int kAdamNT = 256;                           // threads of every Adam workgroup
constexpr int kAdamNF4 = N_PARAMS / 4;                 // 418 float4 = floats 0..1671
constexpr int kAdamNJ = (kAdamNF4 + kAdamNT - 1) / kAdamNT;
static_assert(kAdamNF4 * 4 + 1 == N_PARAMS, "one tail element (lin2.bias[8])");
constexpr int kGradSqBase = SWARM_GRAD_SQ_BASE;     // the norm's group partials in a grad buffer
constexpr int kGradSqCount = SWARM_GRAD_SQ_COUNT;   // 105 groups of 16 parameters
static_assert(kGradSqCount == (N_PARAMS + 15) / 16 && kGradSqCount > 64 && kGradSqCount <= 128, "norm groups");
static_assert(kGradSqBase >= N_PARAMS + 1 && kGradSqBase % 16 == 0 && kGradSqBase + 112 <= SWARM_GRAD_FLOATS,
              "grad buffer layout");
static_assert(kAdamNJ == 2 && kAdamNT == 256, "a thread's float4s i = tid and 256 + tid: groups tid/4 and 64 + tid/4");

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
  float sq_lo, sq_hi;      // the reduce's norm partials sq[lane], sq[lane + 64] (0 past the last)

  // every load issued unconditionally (clamped index): one memory round trip.  partials: also
  // load the slab reduce's norm partials (grad + kGradSqBase)
  __device__ inline void load(const float* __restrict__ grad, const float* __restrict__ w_, const float* __restrict__ m_,
                              const float* __restrict__ v_, int tid, bool partials = false) {
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
    sq_lo = 0.0f; sq_hi = 0.0f;
    if (partials) {
      const int l = tid & 63;
      sq_lo = grad[kGradSqBase + l];
      const float hi = grad[kGradSqBase + min(l + 64, kGradSqCount - 1)];
      sq_hi = l + 64 < kGradSqCount ? hi : 0.0f;
    }
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

// ---- the squared norm in the canonical order (header comment)
// world_size > 1: the summed gradient divided by W first (every path alike)
__device__ inline void adam_scale(AdamRegs& R, const swarm_adam_cfg& hp) {
  if (hp.world_size > 1) {
    const float inv_w = 1.0f / (float)hp.world_size;
#pragma unroll
    for (int j = 0; j < kAdamNJ; ++j) {
      float4 g = R.g[j];
      g.x = g.x * inv_w; g.y = g.y * inv_w; g.z = g.z * inv_w; g.w = g.w * inv_w;
      R.g[j] = g;
    }
    R.gt = R.gt * inv_w;
  }
}
// d[i] of float4 i = tid + 256 j (the tail parameter alone in d[418], 0 past it)
__device__ inline float norm_d(const AdamRegs& R, int j, int tid) {
  const int i = tid + kAdamNT * j;
  const float4 g = R.g[j];
  const float d = ((g.x * g.x + g.y * g.y) + g.z * g.z) + g.w * g.w;
  return i < kAdamNF4 ? d : (i == kAdamNF4 ? R.gt * R.gt : 0.0f);
}
// group sum of a quad of lanes (xor 1, then xor 2): (d0 + d1) + (d2 + d3) in every lane of the quad
__device__ inline float quad_sum(float x) {
  x = x + adam_dpp<0xB1>(x);
  return x + adam_dpp<0x4E>(x);
}
// the block forms the partials from its float4s (one barrier): red >= 64 floats
__device__ inline float adam_norm2_block(const AdamRegs& R, int tid, float* red) {
  const float p = quad_sum(norm_d(R, 0, tid)) + quad_sum(norm_d(R, 1, tid));   // sq[tid/4] + sq[64 + tid/4]
  if ((tid & 3) == 0) red[tid >> 2] = p;
  __syncthreads();
  return wave_sum(red[tid & 63]);
}
// SWARM_ADAM_F_NORM_PARTIALS: every wave from the reduce's partials, no barrier
__device__ inline float adam_norm2_partials(const AdamRegs& R) { return wave_sum(R.sq_lo + R.sq_hi); }

// One optimizer step in registers by the whole workgroup (kAdamNT threads).  step_size /
// inv_bc2_sqrt: ctrl's scalars of this step.  partials: the squared norm from R.sq_lo / sq_hi
// (loaded with partials = true; no barrier), else formed by the block (contains __syncthreads;
// red: LDS scratch of >= 64 floats).  Returns the pre-clip global norm.
template <int SB = -1>   // SB: diagnostic stamp base (SWARM_STAMPS builds only)
// one_m_b1 / one_m_b2: ctrl's (float)(1 - beta) (swarm_ctrl_init, from the double betas): read
// with the control block the prologue loads anyway, not from a kernarg double on its chain
__device__ inline float adam_apply(AdamRegs& R, const swarm_adam_cfg& hp, float step_size, float inv_bc2_sqrt,
                                   float one_m_b1, float one_m_b2, int tid, float* red, bool partials = false) {
#define AD_STAMP(i) do { if (SB >= 0) SWARM_STAMP(SB + (i)); } while (0)
  adam_scale(R, hp);
  AD_STAMP(0);
  // clip_grad_norm_: the norm of the per-tensor norms == the global L2 norm up to rounding
  // (<= ~1e-7 relative on the clip coefficient); one fixed-order reduction
  const float nn = partials ? adam_norm2_partials(R) : adam_norm2_block(R, tid, red);
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
