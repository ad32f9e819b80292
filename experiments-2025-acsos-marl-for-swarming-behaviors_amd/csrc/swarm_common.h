// swarm_common.h — constants, parameter layout, Philox and MFMA helpers shared by
// every kernel of libswarm_hip.so (gfx950 / CDNA4 only).
//
// Arithmetic restated from (paths relative to the reference checkout):
//   VMAS 1.4.0 World.step / scenarios   -> SURVEY.md §8(a) rows a1-a6
//   GCN / PyG GATConv                    -> src/training/train_gcn_dqn.py:50-70
// Every translation unit is compiled with -ffp-contract=off: a*b+c stays two
// roundings unless written as fmaf(), which is what the VMAS/PyTorch CPU path does.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/swarm_hip.h"

namespace swarm {

// ---------------------------------------------------------------- constants
constexpr int kHidden = 32;
constexpr int kFeat = 7;
constexpr int kActions = 9;

constexpr float kGoalX = -0.8f, kGoalY = 0.8f;      // go_to_position_scenario.py:86
constexpr float kObstX = -0.1f, kObstY = 0.1f;      // obstacle_avoidance_scenario.py:99
constexpr float kRadius = 0.05f;                    // VMAS Sphere() default radius
constexpr float kCollisionForce = 100.0f;           // VMAS World collision_force
constexpr float kContactMargin = 0.001f;            // VMAS World contact_margin
constexpr float kMinDist = 1e-6f;                   // VMAS _get_constraint_forces
constexpr float kDt = 0.1f;                         // VMAS dt (substeps = 1)
constexpr float kDragKeep = 0.75f;                  // 1 - drag(0.25)
constexpr float kLeakySlope = 0.2f;                 // GATConv negative_slope
// flocking_scenario.py:10-21: shaping factors, desired spacing, contact threshold, goal bonus
constexpr float kFlockShaping = 10.0f;              // pos_shaping_factor == dist_shaping_factor
constexpr float kFlockDesired = 0.15f;              // desired_distance
constexpr float kFlockContact = 0.005f;             // min_collision_distance
constexpr float kFlockGoalBonus = 50.0f;            // distance_to_goal_reward :146-147

// flat parameter layout == GCN.state_dict() order (see oracle PARAM_ORDER)
constexpr int OFF_ATT_SRC = 0;       // [32]
constexpr int OFF_ATT_DST = 32;      // [32]
constexpr int OFF_BIAS = 64;         // [32]   conv1.bias
constexpr int OFF_W = 96;            // [32][7] conv1.lin.weight
constexpr int OFF_W1 = 320;          // [32][32]
constexpr int OFF_B1 = 1344;         // [32]
constexpr int OFF_W2 = 1376;         // [9][32]
constexpr int OFF_B2 = 1664;         // [9]
constexpr int N_PARAMS = 1673;
constexpr int N_PARAMS_PAD = 1676;   // 16-B multiple (global buffers)
static_assert(OFF_B2 + kActions == N_PARAMS, "param layout");

// LDS weight image: the flat order with every lin1 / lin2 weight row padded to 36
// floats, so MFMA fragment reads (16 rows x 4 columns per instruction) hit 64
// distinct banks.  Float4 chunks of the flat vector never straddle a row.
constexpr int kWRow = 36;
constexpr int L_ATT_SRC = 0;
constexpr int L_ATT_DST = 32;
constexpr int L_BIAS = 64;
constexpr int L_W = 96;
constexpr int L_W1 = 320;                      // [32][36]
constexpr int L_B1 = L_W1 + kHidden * kWRow;   // 1472
constexpr int L_W2 = L_B1 + kHidden;           // 1504, [9][36]
constexpr int L_B2 = L_W2 + kActions * kWRow;  // 1828
constexpr int N_LDS_PARAMS = 1840;             // 16-B multiple
__host__ __device__ constexpr int lds_index(int p) {
  return p < OFF_W1 ? p
       : p < OFF_B1 ? L_W1 + ((p - OFF_W1) >> 5) * kWRow + ((p - OFF_W1) & 31)
       : p < OFF_W2 ? L_B1 + (p - OFF_B1)
       : p < OFF_B2 ? L_W2 + ((p - OFF_W2) >> 5) * kWRow + ((p - OFF_W2) & 31)
       : L_B2 + (p - OFF_B2);
}
static_assert(lds_index(N_PARAMS - 1) == L_B2 + kActions - 1 && L_B2 + kActions <= N_LDS_PARAMS, "LDS image");

// RNG stream ids (third Philox counter word); must match oracle/philox.py
constexpr uint32_t STREAM_COIN = 1;
constexpr uint32_t STREAM_RAND_ACTION = 2;
constexpr uint32_t STREAM_RESET = 3;
constexpr uint32_t STREAM_SAMPLE = 4;

// ---------------------------------------------------------------- Philox4x32-10
struct u32x4 { uint32_t x, y, z, w; };

__host__ __device__ inline u32x4 philox4x32(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                            uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r > 0) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
  }
  return {c0, c1, c2, c3};
}

__host__ __device__ inline float u01(uint32_t w) {   // [0,1), exact in fp32
  return (float)(w >> 8) * 5.9604644775390625e-08f;
}
__host__ __device__ inline int uniform_int(uint32_t w, uint32_t n) {
  return (int)(((uint64_t)w * n) >> 32);
}

// keyed pseudo-random permutation of [0, n): 4-round alternating Feistel network on a
// 2^bits domain whose round function is the lowbias32 integer mixer keyed by one
// Philox block (4 round keys), plus cycle walking (oracle: sample_index).  Cycle
// walking terminates because x lies on a permutation cycle that re-enters [0, n).
__host__ __device__ inline uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}
struct SampleKey { uint32_t rk[4]; int bits; uint32_t n; };
__host__ __device__ inline SampleKey sample_key(uint32_t n, uint32_t k0, uint32_t k1, uint32_t rnd) {
  SampleKey s;
  const u32x4 w = philox4x32(rnd, 0u, STREAM_SAMPLE, 0u, k0, k1);
  s.rk[0] = w.x; s.rk[1] = w.y; s.rk[2] = w.z; s.rk[3] = w.w;
  s.bits = 2;
  while (s.bits < 32 && (1u << s.bits) < n) ++s.bits;
  s.n = n;
  return s;
}
// the key of tick `rnd` from ctrl's cache when its tags match, else derived
__device__ inline SampleKey sample_key_cached(const swarm_ctrl* c, uint32_t n, uint32_t k0, uint32_t k1, uint32_t rnd) {
  if (c->sample_tick == rnd && c->sample_n == n) {
    SampleKey s;
    s.rk[0] = c->sample_key[0]; s.rk[1] = c->sample_key[1]; s.rk[2] = c->sample_key[2]; s.rk[3] = c->sample_key[3];
    s.bits = (int)c->sample_bits;
    s.n = n;
    return s;
  }
  return sample_key(n, k0, k1, rnd);
}
__host__ __device__ inline uint32_t feistel(uint32_t x, const SampleKey& s) {
  const int lo_bits = s.bits / 2, hi_bits = s.bits - lo_bits;
  const uint32_t lo_mask = (1u << lo_bits) - 1u, hi_mask = (1u << hi_bits) - 1u;
  uint32_t L = x >> lo_bits, R = x & lo_mask;
  R ^= mix32(L ^ s.rk[0]) & lo_mask;
  L ^= mix32(R ^ s.rk[1]) & hi_mask;
  R ^= mix32(L ^ s.rk[2]) & lo_mask;
  L ^= mix32(R ^ s.rk[3]) & hi_mask;
  return (L << lo_bits) | R;
}
__host__ __device__ inline uint32_t sample_index(uint32_t i, const SampleKey& s) {
  uint32_t x = i;
  do { x = feistel(x, s); } while (x >= s.n);
  return x;
}
// inverse round order; position of graph id g in the batch permutation (sample_index^-1):
// cycle walking backwards lands on the unique i < n with sample_index(i) == g
__host__ __device__ inline uint32_t feistel_inv(uint32_t y, const SampleKey& s) {
  const int lo_bits = s.bits / 2, hi_bits = s.bits - lo_bits;
  const uint32_t lo_mask = (1u << lo_bits) - 1u, hi_mask = (1u << hi_bits) - 1u;
  uint32_t L = y >> lo_bits, R = y & lo_mask;
  L ^= mix32(R ^ s.rk[3]) & hi_mask;
  R ^= mix32(L ^ s.rk[2]) & lo_mask;
  L ^= mix32(R ^ s.rk[1]) & hi_mask;
  R ^= mix32(L ^ s.rk[0]) & lo_mask;
  return (L << lo_bits) | R;
}
__host__ __device__ inline uint32_t sample_position(uint32_t g, const SampleKey& s) {
  uint32_t x = g;
  do { x = feistel_inv(x, s); } while (x >= s.n);
  return x;
}

// ---------------------------------------------------------------- gradient slabs
// Each TD block writes its partial gradient (N_PARAMS + 1 columns, the last the loss sum) as a
// slab; the reduce launch sums column block j (16 columns) over all slabs in block order.
// Layout: column-block major, [kSlabColBlocks][n_slabs][16], so one reduce block reads one
// contiguous n_slabs x 64 B run (whole 128-B lines, each fetched by one block) instead of a
// 64-B piece of every 6.7-KB slab row.
constexpr int kSlabCols = 16;
constexpr int kSlabColBlocks = (N_PARAMS + 1 + kSlabCols - 1) / kSlabCols;
__host__ __device__ constexpr size_t slab_floats_per_block() { return (size_t)kSlabColBlocks * kSlabCols; }
__host__ __device__ inline size_t slab_index(int q, int b, int n_slabs) {
  return ((size_t)(q / kSlabCols) * n_slabs + b) * kSlabCols + (q % kSlabCols);
}

// ---------------------------------------------------------------- fused-tick hand-off
// The fused training tick (swarm_tick.hip) runs the acting blocks beside the TD blocks.
// A TD graph drawn from THIS tick's replay slot is the transition an acting wave is still
// producing: that wave publishes it as tagged granules — 8 bytes {tag = tick + 1, value},
// each ONE aligned write-through (sc1) store — into an env-exclusive record (whole 128-B
// lines); the TD wave re-reads its granules with sc1 loads until every tag matches, so
// the data is its own flag: no producer drain, no flag, no second round trip
// (cdna_hip_programming.md §6 Guideline 16, R2).  Tags never repeat (the tick counter
// advances every tick), so no per-launch reset is needed.
// Record of env e (granule index): s [N][4] at 4n + k, s' [N][4] at 4N + 4n + k, r at 8N + n,
// a at 9N + n.
__host__ __device__ constexpr int ho_stride_granules(int N) { return ((10 * N + 15) / 16) * 16; }
// Through global-address-space pointers: the TD waves' polls read the record through a pointer
// the compiler cannot trace to a kernel argument, so they were flat loads, which count in lgkmcnt
// as well as vmcnt (a wait for a poll then also drained the wave's LDS operations, and an LDS
// wait the poll).  As global loads they count in vmcnt only
typedef __attribute__((address_space(1))) unsigned long long gran_t;
__device__ inline void st_granule(unsigned long long* g, uint32_t tag, uint32_t value) {
  __hip_atomic_store((gran_t*)g, ((unsigned long long)tag << 32) | value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline unsigned long long ld_granule(const unsigned long long* g) {
  return __hip_atomic_load((const gran_t*)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One 16-B write-through store (global_store_dwordx4 ... sc1): the line leaves the XCD's L2 as it
// is written, so a launch that ends after it leaves no dirty line behind for the end-of-kernel
// write-back (MI355X_MICROARCH.md "boundary": + bytes / 6 TB/s), and a 16-B sc1 store costs what a
// plain one does.  Inline asm is invisible to the compiler's hazard recognizer: the data may be
// MFMA results, which a vector-memory instruction may read only after the MFMA's wait states (not
// interlocked; without the padding a store read partial sums, profiles/r06_bitcmp_b2t_v1.jsonl),
// so 24 wait states lead the store.  Vector store only (never a scalar-cache write).
__device__ inline void st16_wt(float* p, float a, float b, float c, float d) {
  typedef float f4v __attribute__((ext_vector_type(4)));
  const f4v x = {a, b, c, d};
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\tglobal_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(x) : "memory");
}

// ---------------------------------------------------------------- small math
__host__ __device__ inline float leaky(float x) { return x > 0.0f ? x : x * kLeakySlope; }

// tanh from one v_exp_f32 and one v_rcp_f32: t = sign(x) (1 - 2 / (exp(2|x|) + 1)).
// |error| <= ~3e-7 absolute against torch.tanh (checked by the Q-value parity tests);
// ocml tanhf costs ~230 cycles per call on the single-wave critical path.
__device__ inline float tanh_fast(float x) {
  const float e = __expf(2.0f * fabsf(x));
  const float t = 1.0f - 2.0f * __builtin_amdgcn_rcpf(e + 1.0f);
  return copysignf(t, x);
}

// torch.linalg.vector_norm of a 2-vector on CPU == sqrtf(fmaf(dy, dy, dx*dx))
// (re-checked by tests/test_knn_host.py against torch).
__host__ __device__ inline float norm2(float dx, float dy) { return sqrtf(fmaf(dy, dy, dx * dx)); }

// torch.logaddexp(0, x) CPU scalar path: max(0,x) + log1p(exp(-|x|))
__device__ inline float logaddexp0(float x) {
  const float m = x > 0.0f ? x : 0.0f;
  return m + log1pf(expf(-fabsf(x)));
}

// VMAS _get_constraint_forces (attractive = False): force on entity a of the
// pair (a, b) with delta = p_a - p_b; force on b is the exact negation.
// Pairs out of contact (dist > r_a + r_b) or coincident (dist < 1e-6) get exactly 0,
// as the two torch.where of the reference do, so the transcendental part is skipped.
// In two pieces so that a wave can test every pair first and evaluate only the pairs in contact
// (swarm_actk.h pair_forces): the same operations in the same order as one call.
__device__ inline bool pair_contact(float dist) { return !(dist < kMinDist || dist > kRadius + kRadius); }
__device__ inline void contact_force(float dx, float dy, float dist, float& fx, float& fy) {
  const float dmin = kRadius + kRadius;
  const float pen = logaddexp0((dmin - dist) / kContactMargin) * kContactMargin;
  const float den = dist > 0.0f ? dist : 1e-8f;
  fx = kCollisionForce * dx / den * pen;
  fy = kCollisionForce * dy / den * pen;
}
__device__ inline void pair_force(float dx, float dy, float& fx, float& fy) {
  const float dist = norm2(dx, dy);
  fx = 0.0f;
  fy = 0.0f;
  if (!pair_contact(dist)) return;
  contact_force(dx, dy, dist, fx, fy);
}

// discrete action a in 0..8 -> u = (L[a/3], L[a%3]), L = {0, -1, +1}  
__host__ __device__ inline float action_level(int l) { return l == 0 ? 0.0f : (l == 1 ? -1.0f : 1.0f); }

// ---------------------------------------------------------------- diagnostic stamps
// Built only into the diagnostic libraries; lane 0 of every wave records a clock at named
// points into the buffer swarm_dbg_stamps_* installs:
//  - SWARM_STAMPS=1 (libswarm_hip_stamps.so): s_memtime segment stamps (SWARM_STAMP) and the
//    s_memrealtime launch stamps (SWARM_RTSTAMP); read the SHARES, never that build's run time
//    (cdna_hip_programming.md §7 "In-kernel stamps");
//  - SWARM_STAMPS=2 (libswarm_hip_rtstamps.so): the realtime launch stamps only (a few per wave),
//    for kernel spans and launch boundaries close to the product build's (tools/tick_split_stamps.py).
#ifndef SWARM_STAMPS
#define SWARM_STAMPS 0
#endif
#if SWARM_STAMPS
static __constant__ unsigned long long* g_swarm_stamps;
#define SWARM_STAMP_AT(k, instr)                                                              \
  do {                                                                                        \
    __builtin_amdgcn_sched_barrier(0);                                                        \
    unsigned long long _t;                                                                    \
    asm volatile(instr " %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");                  \
    __builtin_amdgcn_sched_barrier(0);                                                        \
    if (g_swarm_stamps && (threadIdx.x & 63) == 0)                                            \
      g_swarm_stamps[((size_t)blockIdx.x * 16 + (threadIdx.x >> 6)) * 32 + (k)] = _t;         \
  } while (0)
// s_memrealtime: the chip-wide 100 MHz clock, comparable across XCDs (launch spans, gaps)
#define SWARM_RTSTAMP(k) SWARM_STAMP_AT(k, "s_memrealtime")
#endif
#if SWARM_STAMPS == 1
#define SWARM_STAMP(k) SWARM_STAMP_AT(k, "s_memtime")
#else
#define SWARM_STAMP(k) \
  do {              \
  } while (0)
#endif
#if !SWARM_STAMPS
#define SWARM_RTSTAMP(k) \
  do {                \
  } while (0)
#endif

// compile-time graph / conv specialisations of the act and TD kernels
// (SPEC_RADIUS_GAT: the north_star's radius-neighbour graph, GoTo training ticks of <= 8 agents)
enum { SPEC_RUNTIME = 0, SPEC_COMPLETE_GAT = 1, SPEC_COMPLETE_GCN = 2, SPEC_KNN_GAT = 3, SPEC_RADIUS_GAT = 4 };
__host__ __device__ inline int spec_of(int graph, int conv) {
  if (graph == SWARM_GRAPH_COMPLETE) return conv == SWARM_CONV_GAT ? SPEC_COMPLETE_GAT : SPEC_COMPLETE_GCN;
  if (graph == SWARM_GRAPH_KNN && conv == SWARM_CONV_GAT) return SPEC_KNN_GAT;
  if (graph == SWARM_GRAPH_RADIUS && conv == SWARM_CONV_GAT) return SPEC_RADIUS_GAT;
  return SPEC_RUNTIME;
}
template <int SPEC>
__device__ inline int spec_graph(int runtime) {
  return SPEC == SPEC_RUNTIME       ? runtime
         : SPEC == SPEC_KNN_GAT     ? (int)SWARM_GRAPH_KNN
         : SPEC == SPEC_RADIUS_GAT  ? (int)SWARM_GRAPH_RADIUS
                                    : (int)SWARM_GRAPH_COMPLETE;
}
template <int SPEC>
__device__ inline int spec_conv(int runtime) {
  return SPEC == SPEC_RUNTIME ? runtime : (SPEC == SPEC_COMPLETE_GCN ? (int)SWARM_CONV_GCN : (int)SWARM_CONV_GAT);
}

}  // namespace swarm
