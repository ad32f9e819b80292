// swarm_tdk.h — body of the TD kernel: replay sample, TD loss, hand-written backward
// through GCN (PyG GATConv + MLP), per-block gradient slabs.  Shared by td_kernel
// (swarm_td.hip) and the fused training-tick kernel (swarm_tick.hip).
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
// MFMA (16x16x4 f32 tiles, node index as K), vectors by LDS column sums; each block writes one
// slab [N_PARAMS + 1] (last = sum of squared TD errors) and swarm_grad_reduce sums the
// slabs in a fixed order (bitwise run-to-run reproducible).
#pragma once
#include "swarm_adam.h"
#include "swarm_dl.h"

namespace swarm {

// One TD block = 32 node slots = GPB = 32 / NS sampled graphs.  Wave w < GPB runs the
// ONLINE network on graph w (forward on s with activations kept, dQ, backward of the
// per-node vectors); wave GPB + w runs the TARGET network on s' of graph w
// (y = r + gamma max_a Q_tgt), then shares the parameter products.  The parameter
// gradient of the block is a sum over its 32 node rows: MFMA 16x16x4 f32 tiles with the
// node index as K, spread over the waves, each writing its slice of the slab.
constexpr int kTdRows = 32;

template <int NS>
struct TdLds {
  static constexpr int GPB = kTdRows / NS;
  float H[kTdRows][kRow];         // online conv1.lin output
  float T[kTdRows][kRow];         // tanh(conv out)
  float R[kTdRows][kRow];         // relu(lin1)
  // written only after B1; before it, rows NS w .. NS w + NS - 1 of dZ / dO / dH are target
  // wave w's forward scratch (its H / T / R rows): 13.8 KB less LDS per block, so three
  // 256-thread blocks fit a CU (the fused tick at N = 9..16 has 3 blocks per CU)
  float dZ[kTdRows][kRow];        // dL/d lin1 pre-activation
  float dO[kTdRows][kRow];        // dL/d conv out
  float dH[kTdRows][kRow];        // dL/d h
  float X[kTdRows][9];            // node features (k < 8)
  union {
    struct {
      float cm[kTdRows][NS + 1];  // c[target row][source slot]
      float dp[kTdRows][NS + 1];  // dL/d pre-activation of edge (source -> target row)
    };
    WSmall<NS> tgsm[GPB];         // before B1: the target waves' small scratch
  };
  float yq[kTdRows], gq[kTdRows], das[kTdRows], dad[kTdRows], d2[kTdRows];   // yq: gamma max_a Q_target(s')
  int act[kTdRows];
  int tdrop[kTdRows];             // fused tick: the target wave dropped this row's graph (hand-off overrun)
  int prew[GPB];                  // online wave w is on the pre path (swarm_tdk.h td_body)
  int insl[GPB];                  // before B0: online wave w holds a graph of this tick's slot
  WSmall<NS> on[GPB];             // online waves' per-graph scratch
  __device__ WView<NS> target_view(int w) { return WView<NS>{dZ + NS * w, dO + NS * w, dH + NS * w, &tgsm[w]}; }
};

struct TdArgs {
  int S, B, N, graph, k, conv, env_offset;
  uint32_t k0, k1;
  float radius;
  const float* params;
  const float* target;
  swarm_replay replay;
  const swarm_ctrl* ctrl;
  const int32_t* sample_in;
  int32_t* sample_out;
  float* slabs;
  float gamma;
  float grad_scale;   // fp32(2 / M_local)
  int n_slabs;        // TD blocks of the launch (slab layout, swarm_common.h slab_index)
};

// gradient-slab store (read once by the next launch, from another XCD).  The 4-B stores stay plain:
// as nt (td 8.4 vs 8.0 us) and as 4-B write-through sc1 (9.5 us; round 6 again: +0.1-0.2 us per
// tick) they cost more; the dW1 / dW2 tiles' 16-B pieces are write-through (sst4)
__device__ inline void slab_st(float* p, float v) { *p = v; }
#ifndef SWARM_DIAG_FEWSLABS
#define SWARM_DIAG_FEWSLABS 0   // diagnostic builds only: > 0 = only the first K TD blocks store slabs (timing bound)
#endif

// NS node slots per wave holding NS / GS graphs of GS slots (GS = 8 < NS = 16 packs two
// N <= 8 graphs into one wave: every MFMA column is a real node, one wave per SIMD).
// The dependent chain's pointers (batch indices -> replay rows) and the geometry lead the
// parameter list: preloaded into SGPRs (kernarg preload), the index loads issue at wave start.
template <int NS>
struct TdSmem {
  TdLds<NS> TB;
  __attribute__((aligned(16))) float Pon[N_LDS_PARAMS];
  __attribute__((aligned(16))) float Ptg[N_LDS_PARAMS];
  float red[64];   // fused tick: the optimizer step's norm (adam_norm2_block)
};

// the TD half of the fused training tick (swarm_tick.hip): weights from the pending
// optimizer step (recomputed in registers, as every acting block does), batch indices
// drawn in-kernel, this tick's slot read from the acting waves' hand-off records
struct TdFused {
  swarm_learner lr;
  swarm_adam_cfg hp;
  const unsigned long long* ho_rec;   // [B][ho_stride_granules(N)] tagged hand-off records
  uint32_t* ho_err;                   // bounded-wait overruns (0 in a correct run)
};
#ifndef SWARM_HO_SPIN_LIMIT
#define SWARM_HO_SPIN_LIMIT (1 << 18)
#endif
#ifndef SWARM_HO_FORCE_DROP
#define SWARM_HO_FORCE_DROP 0
#endif
#ifndef SWARM_HO_SLEEP
#define SWARM_HO_SLEEP 1  // s_sleep argument (x 64 cycles) between two hand-off sweeps
#endif
constexpr int kHoSpinLimit = SWARM_HO_SPIN_LIMIT;   // polls (with s_sleep) before a hand-off wait gives up
// test builds only (libswarm_hip_hodrop.so): every hand-off wait overruns at once
constexpr bool kHoForceDrop = SWARM_HO_FORCE_DROP == 1;
// test builds only (libswarm_hip_hodrop2.so): the target waves' s' waits overrun at once and the
// online waves never see r (their waits run to the bound): an overrun counts once per wave that
// dropped, not again in the online wave's r wait for a graph its target wave already dropped
constexpr bool kHoDropTarget = SWARM_HO_FORCE_DROP == 2;

// A hand-off wait that overruns drops the graphs it waited for: their nodes become padding
// (no TD error, no gradient, no loss), so the update is the mean over the S*N batch nodes with
// those graphs' terms zero, never one computed from a stale granule.  The overrun is counted in
// the workspace's error word (SwarmEngine.handoff_errors; DQNTrainer raises on it).  Node slot
// 16 ct + c belongs to graph (16 ct + c) / GS: with GS < 16 the lanes of its column group
// (c / GS, all four row groups) in one ct; GS = 16 one whole ct; GS = 32 both.
template <int NS, int GS>
__device__ inline void drop_overrun(const bool (&okc)[DGeom<NS>::CT], bool (&drop)[DGeom<NS>::CT],
                                    bool (&nv)[DGeom<NS>::CT], int c) {
  constexpr int CT = DGeom<NS>::CT;
  bool bad[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    const unsigned long long m = __builtin_amdgcn_ballot_w64(!okc[ct]);
    if constexpr (GS < 16) {
      const unsigned long long cols = (((1ull << GS) - 1ull) << (GS * (c / GS))) * 0x0001000100010001ull;
      bad[ct] = (m & cols) != 0ull;
    } else {
      bad[ct] = m != 0ull;
    }
  }
  if constexpr (GS > 16) {   // one graph over every ct of the wave
    bool any = false;
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) any = any || bad[ct];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) bad[ct] = any;
  }
#pragma unroll
  for (int ct = 0; ct < CT; ++ct)
    if (bad[ct]) { drop[ct] = true; nv[ct] = false; }
}

template <int NS, int GS, int SPEC, bool FUSED = false>   // SPEC: graph + conv fixed at compile time (swarm_common.h)
__device__ __forceinline__ void td_body(TdSmem<NS>& L, const int vb, const int32_t* sample_in, const float* rs,
                                        const float* rs_next, const float* rr, const uint8_t* ra, int S, int B,
                                        int N, int capacity, const TdArgs& A, const TdFused& X,
                                        const swarm_ctrl* __restrict__ ctrl_pre = nullptr, const float* g_pre = nullptr,
                                        const float* w_pre = nullptr, const float* m_pre = nullptr,
                                        const float* v_pre = nullptr) {
  constexpr int GPB = kTdRows / NS, CT = DGeom<NS>::CT;   // GPB: online (= target) waves per block
  constexpr int GPW = NS / GS;                             // graphs per wave
  constexpr int NT = 128 * GPB;
  static_assert(!FUSED || NT == kAdamNT, "the fused TD block is one Adam workgroup");
  static_assert(GPB <= 2, "B2 jobs 2 and 3 go to the pre-path online waves by wave index (GPB <= 2)");
  TdLds<NS>& TB = L.TB;
  float* Pon = L.Pon;
  float* Ptg = L.Ptg;
  const int wave = threadIdx.x >> 6;
  const bool online = wave < GPB;
  const int wi = online ? wave : wave - GPB;
  const DGeom<NS> d = make_dgeom<NS>(vb * GPB + wi, 1 << 30);   // lane geometry; liveness is per graph
  const int graph = spec_graph<SPEC>(A.graph);
  const int conv = spec_conv<SPEC>(A.conv);
  const int row0 = wi * NS;
  const WView<NS> V = online ? WView<NS>{TB.H + row0, TB.T + row0, TB.R + row0, &TB.on[wi]} : TB.target_view(wi);
  const int lane = d.lane, c = d.c, p = d.p;
  // this block's slab column q (swarm_common.h slab_index: column-block major), addressed as a
  // wave-uniform base (the block's 16-column run in column block 0) plus a 32-bit element
  // offset: one 64-bit add per block instead of 64-bit index arithmetic per store
  static_assert(kSlabCols == 16, "slab column blocks of 16");
  float* const slab_base = A.slabs + (size_t)vb * kSlabCols;
  const uint32_t slab_stride = (uint32_t)A.n_slabs * kSlabCols;
#if SWARM_DIAG_FEWSLABS > 0
  auto sst_g = [&](int q, float v) {
    if (vb < SWARM_DIAG_FEWSLABS) slab_st(slab_base + ((uint32_t)(q >> 4) * slab_stride + (uint32_t)(q & 15)), v);
  };
#elif SWARM_DIAG_FEWSLABS < 0   // -1: blocks holding a graph of this tick's slot skip their stores; -2: the others do
  bool diag_skip = false;   // set once the block knows whether it holds such a graph
  auto sst_g = [&](int q, float v) {
    if (!diag_skip) slab_st(slab_base + ((uint32_t)(q >> 4) * slab_stride + (uint32_t)(q & 15)), v);
  };
#else
  auto sst_g = [&](int q, float v) { slab_st(slab_base + ((uint32_t)(q >> 4) * slab_stride + (uint32_t)(q & 15)), v); };
#endif
// the dW1 / dW2 tiles' 16-B pieces: four consecutive parameters q .. q + 3 (q % 4 == 0) of one
// 16-column slab run, stored write-through (swarm_common.h st16_wt): the 1,312 of a slab's 1,674
// floats leave the XCD's L2 as they are written instead of at the launch end (round 6: C2 -0.22,
// C3 -0.43 us per tick, profiles/r06_ab_b2t_v3_*.jsonl; plain 16-B stores were neutral)
  static_assert(OFF_W1 % 16 == 0 && OFF_W2 % 16 == 0 && kHidden % 16 == 0, "16-B slab pieces");
  auto sst4 = [&](int q, f32x4 v) {
#if SWARM_DIAG_FEWSLABS > 0
    if (vb >= SWARM_DIAG_FEWSLABS) return;
#elif SWARM_DIAG_FEWSLABS < 0
    if (diag_skip) return;
#endif
    st16_wt(slab_base + ((uint32_t)(q >> 4) * slab_stride + (uint32_t)(q & 15)), v[0], v[1], v[2], v[3]);
  };
  auto sst = sst_g;
  SWARM_RTSTAMP(8);
  SWARM_STAMP(0);

  // ---- 3-launch tick: this wave's replay indices come from the previous launch, so the
  //      dependent pair (index -> replay rows) is issued first and the weight staging and
  //      ctrl reads overlap it.  Indices are clamped into the ring: a skipped tick reads
  //      valid (unused) rows.  Fused tick: the pending Adam step's operands and ctrl first.
  AdamRegs R;
  swarm_ctrl cc = {};
  if (FUSED) {   // the fused kernel's preloaded argument SGPRs (== X.lr / A.ctrl): no kernarg round trip first
    cc = *ctrl_pre;   // issued before any kernarg-segment load, so no wait on one delays it
    __builtin_amdgcn_sched_barrier(0);
    R.load(g_pre, w_pre, m_pre, v_pre, threadIdx.x, true);
    __builtin_amdgcn_sched_barrier(0);   // every Adam operand load issued before the first scalar wait
  }
  // fused: the scalars the sampling, the hand-off test and the optimizer step read (ctrl's
  // write_slot, the batch size S, the Adam hyper-parameters) made opaque here, so they are
  // loaded with the first scalar wait instead of being re-fetched at a later first use behind a
  // second one (a kernarg / ctrl round trip on the TD chain)
  swarm_adam_cfg hp = X.hp;
  int32_t* sample_out = A.sample_out;
  const unsigned long long* ho_rec = X.ho_rec;
  if (FUSED) {
    asm volatile("" : "+s"(cc.write_slot), "+s"(cc.trained), "+s"(S), "+s"(hp.beta1), "+s"(hp.beta2), "+s"(hp.eps),
                 "+s"(hp.max_norm), "+s"(hp.update_target_every), "+s"(hp.world_size), "+s"(sample_out), "+s"(ho_rec));
  }
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
    sid[ct] = vb * (kTdRows / GS) + wi * GPW + gi;
    live[ct] = sid[ct] < S && n < NS;
    nv[ct] = live[ct] && jl[ct] < N;
    gid[ct] = 0;
    if (!FUSED && sample_in) gid[ct] = min((uint32_t)sample_in[min(sid[ct], S - 1)], ring_graphs - 1u);
  }
  ParamStage<NT> pon, ptg;
  if (!FUSED) pon.load(A.params, threadIdx.x);
  ptg.load(A.target, threadIdx.x);   // fused: overridden by the new weights on a sync tick
  const uint32_t filled = FUSED ? cc.filled_slots : A.ctrl->filled_slots;
  const uint32_t valid_slots = filled + 1 < cap ? filled + 1 : cap;
  const uint32_t n_graphs = valid_slots * (uint32_t)B;
  if (FUSED || !sample_in) {   // GraphReplayBuffer.sample: random.sample -> keyed permutation
    const uint32_t k0 = A.k0 ^ ((uint32_t)A.env_offset * 0x9E3779B9u);
    const SampleKey sk = FUSED ? sample_key_cached(&cc, n_graphs, k0, A.k1, cc.tick)
                               : sample_key(n_graphs, k0, A.k1, A.ctrl->tick);
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
      gid[ct] = n_graphs >= (uint32_t)S ? sample_index((uint32_t)min(sid[ct], S - 1), sk) : 0u;
  }
  // graphs of this tick's slot (fused: they come from the acting waves' hand-off records).  A
  // wave holding one takes the pre path in every kind of launch (fused, 3-launch, unfused), so
  // the three stay bit-identical to each other
  const uint32_t wslot = FUSED ? cc.write_slot : A.ctrl->write_slot;
  bool ho[CT];
  bool wait = false, inslot = false;
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    const bool cur = live[ct] && n_graphs >= (uint32_t)S && gid[ct] / (uint32_t)B == wslot;
    ho[ct] = FUSED && cur;
    wait = wait || ho[ct];
    inslot = inslot || cur;
  }
  // replay rows written by earlier ticks: loads issued now (fused: every lane but the hand-off ones)
  float rew[CT];
  int act[CT];
  float4 st[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    const uint32_t slot = gid[ct] / (uint32_t)B, genv = gid[ct] % (uint32_t)B;
    const size_t ri = ((size_t)slot * B + genv) * N + min(jl[ct], N - 1);
    st[ct] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    rew[ct] = 0.0f;
    act[ct] = 0;
    if (!ho[ct]) {
      st[ct] = reinterpret_cast<const float4*>(online ? rs : rs_next)[ri];
      rew[ct] = rr[ri];
      act[ct] = nv[ct] ? (int)ra[ri] : 0;
    }
  }
  // ---- skip while the replay holds fewer than `batch` graphs (train_gcn_dqn.py:113-115)
  if (n_graphs < (uint32_t)S) {
    for (int q = threadIdx.x; q <= N_PARAMS; q += NT) sst_g(q, 0.0f);
    return;
  }
  if (sample_out && online && p == 0) {
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
      if (live[ct] && jl[ct] == 0) sample_out[sid[ct]] = (int32_t)gid[ct];
  }
  SWARM_STAMP(1);
  const bool waited = FUSED && __builtin_amdgcn_ballot_w64(wait) != 0;
  // pre path: the online waves of a block holding one of this tick's transitions form their
  // backward for gq = 1 before y (dZ, dT, dO, the attention scores' g and dp are linear in their
  // target node's gq; the sums that mix targets, da_src and dh, stay after B2), in the time the
  // block waits for the acting wave's s' and the target forward.  Every online wave of such a
  // block takes it (round 4): the one without a hand-off graph otherwise ran its whole backward
  // after B1 and was the last to reach B3.  The rule depends only on the block's graphs, so the
  // fused, 3-launch and unfused launches still agree bit for bit
  if (online && lane == 0) TB.insl[wi] = __builtin_amdgcn_ballot_w64(inslot) != 0 ? 1 : 0;
  bool live_drop[CT];   // this wave's graph was dropped after a hand-off overrun
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) live_drop[ct] = false;
  if (FUSED) {   // the pending optimizer step (train_gcn_dqn.py:125-133), as every acting block does;
                 // done before any hand-off wait so that none of it follows the wait
    const bool pending = cc.trained != 0u && cc.peer_hold == 0u;   // a held rank applies no step
    if (pending)
      adam_apply(R, hp, cc.adam_step_size, cc.adam_inv_bc2, cc.one_m_beta1, cc.one_m_beta2, threadIdx.x, L.red,
                 (hp.flags & SWARM_ADAM_F_NORM_PARTIALS) != 0);
    store_w_lds(Pon, R, threadIdx.x);
    if (pending && (cc.tick % (uint32_t)hp.update_target_every) == 0u) store_w_lds(Ptg, R, threadIdx.x);
    else ptg.store(Ptg, threadIdx.x);
  } else {
    pon.store(Pon, threadIdx.x);
    ptg.store(Ptg, threadIdx.x);
  }
  if (online && p == 0 && !waited) {
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
      if (16 * ct + c < NS) TB.act[row0 + 16 * ct + c] = act[ct];
  }
  if (FUSED && !online && p == 0) {   // no graph dropped yet (set by an s' overrun, read by the r wait)
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
      if (16 * ct + c < NS) TB.tdrop[row0 + 16 * ct + c] = 0;
  }
  __syncthreads();   // B0: weight images
  SWARM_STAMP(2);
  bool pre = false;
#pragma unroll
  for (int w2 = 0; w2 < GPB; ++w2) pre = pre || TB.insl[w2] != 0;
#if SWARM_DIAG_PRE_ALL   // diagnostic builds only (tools/ab_build.py): every block on the pre path
  pre = true;
#endif
#if SWARM_DIAG_FEWSLABS < 0
  diag_skip = (SWARM_DIAG_FEWSLABS == -1) == pre;
#endif
  pre = pre && online;
  const uint32_t tag = cc.tick + 1u;
  // granule address of this lane's node in a hand-off record: s at 0, s' at 4N, r at 8N, a at 9N
  auto ho_at = [&](int ct, int off, int per_node) -> const unsigned long long* {
    return ho_rec + (size_t)(gid[ct] % (uint32_t)B) * ho_stride_granules(N) + off + per_node * min(jl[ct], N - 1);
  };
  if (waited) {   // sweep this lane's granules until every tag is this tick's (R2 hand-off): online
                  // waves s (published at the acting prologue), target waves s' (after the integrator).
                  // Wave-local, after B0: the block's other waves are not held by it
    for (int spin = 0;; ++spin) {
      unsigned long long g[CT][4];
#pragma unroll
      for (int ct = 0; ct < CT; ++ct)
        if (ho[ct]) {
          const unsigned long long* sp = ho_at(ct, online ? 0 : 4 * N, 4);
#pragma unroll
          for (int k = 0; k < 4; ++k) g[ct][k] = ld_granule(sp + k);
        }
      bool ok = true, okc[CT];
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        okc[ct] = true;
        if (ho[ct]) {
          okc[ct] = !kHoForceDrop && !(kHoDropTarget && !online) && (uint32_t)(g[ct][0] >> 32) == tag &&
                    (uint32_t)(g[ct][1] >> 32) == tag && (uint32_t)(g[ct][2] >> 32) == tag &&
                    (uint32_t)(g[ct][3] >> 32) == tag;
          ok = ok && okc[ct];
          st[ct] = make_float4(__uint_as_float((uint32_t)g[ct][0]), __uint_as_float((uint32_t)g[ct][1]),
                               __uint_as_float((uint32_t)g[ct][2]), __uint_as_float((uint32_t)g[ct][3]));
        }
      }
      if (!__builtin_amdgcn_ballot_w64(!ok)) break;
      if (kHoForceDrop || (kHoDropTarget && !online) || spin >= kHoSpinLimit) {   // never in a correct
        drop_overrun<NS, GS>(okc, live_drop, nv, c);                              // run: drop, count
        // tell the online waves' r wait first (they then drop without counting again), count after.
        // An online wave whose own r wait overruns BEFORE this store counts the graph as well: the
        // error word counts dropping waves, and is nonzero whenever a graph was dropped
        if (FUSED && !online && p == 0) {
#pragma unroll
          for (int ct = 0; ct < CT; ++ct)
            if (16 * ct + c < NS && live_drop[ct]) *(volatile int*)&TB.tdrop[row0 + 16 * ct + c] = 1;
        }
        if (lane == 0) atomicAdd(X.ho_err, 1u);
        break;
      }
      __builtin_amdgcn_s_sleep(SWARM_HO_SLEEP);
    }
    SWARM_RTSTAMP(10);
    __builtin_amdgcn_s_setprio(3);   // waves of hand-off graphs are the tick's critical path
  }
  DFwd<NS> F;
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    node_x(st[ct].x, st[ct].y, st[ct].z, st[ct].w, jl[ct], p, F.x[ct]);
    if (!nv[ct]) { F.x[ct][0] = 0.0f; F.x[ct][1] = 0.0f; }
  }
  // ---- forwards: online on s (activations kept), target on s' (train_gcn_dqn.py:119-121).
  //      Everything after B1 waits for the target waves' y, so they issue first.
  if (!online && !waited) __builtin_amdgcn_s_setprio(2);
  dl_forward<NS, 16, GS>(online ? Pon : Ptg, d, N, graph, A.k, A.radius, conv, nullptr, V, online, F);
  // fused: the rest of this tick's transitions, each as late as its first use: a for the online
  // waves' pre path here; r (published after the acting wave's reward) by the online waves after
  // it, in their wait for the target waves' y, so no poll sits between the target forward and B1
  if (FUSED && waited && online) {
    for (int spin = 0;; ++spin) {
      bool ok = true, okc[CT];
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        okc[ct] = true;
        if (ho[ct] && !live_drop[ct]) {
          const unsigned long long g = ld_granule(ho_at(ct, 9 * N, 1));
          okc[ct] = !kHoForceDrop && (uint32_t)(g >> 32) == tag;
          ok = ok && okc[ct];
          act[ct] = nv[ct] ? (int)(uint32_t)g : 0;
        }
      }
      if (!__builtin_amdgcn_ballot_w64(!ok)) break;
      if (kHoForceDrop || spin >= kHoSpinLimit) {
        if (lane == 0) atomicAdd(X.ho_err, 1u);
        drop_overrun<NS, GS>(okc, live_drop, nv, c);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (p == 0) {
#pragma unroll
      for (int ct = 0; ct < CT; ++ct)
        if (16 * ct + c < NS) TB.act[row0 + 16 * ct + c] = nv[ct] ? act[ct] : 0;
    }
  }
  // ---- pre path, before y: dZ1 = W2[a] * [z > 0], dO1 = (W1^T dZ1) (1 - t^2) (MFMA, as after B2),
  //      g1 = H_u . dO1_v, dp1 / da_dst1 of the attention (scaled by gq after B1)
  float dO1[CT][2][4], dp1[CT][CT][4], dad1[CT];
  if (pre) {
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      const int ac = min(max(act[ct], 0), kActions - 1);
      float dz1[2][4];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const float4 w = *reinterpret_cast<const float4*>(Pon + L_W2 + ac * kWRow + 16 * t + 4 * p);
        float wv[4] = {w.x, w.y, w.z, w.w};
        asm volatile("" : "+v"(wv[0]), "+v"(wv[1]), "+v"(wv[2]), "+v"(wv[3]));
#pragma unroll
        for (int r = 0; r < 4; ++r) dz1[t][r] = F.zr[ct][t][r] > 0.0f ? wv[r] : 0.0f;
      }
      float w1f[2][2][4];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int t2 = 0; t2 < 2; ++t2) w1f[t2][t][r] = Pon[L_W1 + (16 * t + 4 * p + r) * kWRow + 16 * t2 + c];
      f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int t2 = 0; t2 < 2; ++t2) acc[t2] = mfma16(w1f[t2][t][r], dz1[t][r], acc[t2]);
#pragma unroll
      for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
        for (int r = 0; r < 4; ++r) dO1[ct][t2][r] = acc[t2][r] * (1.0f - F.t[ct][t2][r] * F.t[ct][t2][r]);
      dad1[ct] = 0.0f;
#pragma unroll
      for (int ut = 0; ut < CT; ++ut)
#pragma unroll
        for (int r = 0; r < 4; ++r) dp1[ct][ut][r] = 0.0f;
    }
    if (conv == SWARM_CONV_GAT) {
      const WSmall<NS>& sm = *V.sm;
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
        float gv[CT][4], cu[CT][4];
        float part = 0.0f;
#pragma unroll
        for (int ut = 0; ut < CT; ++ut) {
          f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc = mfma16(ah[ut][t][r], dO1[ct][t][r], acc);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float cc4[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int uq = 16 * ut + 4 * q + r;
              cc4[q] = uq < NS ? F.cf[ct][uq < NS ? uq : 0] : 0.0f;
            }
            cu[ut][r] = p == 0 ? cc4[0] : (p == 1 ? cc4[1] : (p == 2 ? cc4[2] : cc4[3]));
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
            if (u < NS && cu[ut][r] != 0.0f) {   // in-edges only (cross-graph / absent: c = 0)
              const float de = cu[ut][r] * (gv[ut][r] - Gs);
              const float pre_act = sm.ssrc[u] + F.sdst[ct];
              dpu = pre_act > 0.0f ? de : de * kLeakySlope;
            }
            dsum = dsum + dpu;
            dp1[ct][ut][r] = dpu;
          }
        dad1[ct] = row4_sum(dsum);
      }
    }
  }
  if (FUSED && waited && online) {   // r of this tick's transitions (y = r + gamma max Q_tgt after B1)
    for (int spin = 0;; ++spin) {
      bool ok = true, okc[CT];
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        okc[ct] = true;
        if (ho[ct] && !live_drop[ct]) {
          const unsigned long long g = ld_granule(ho_at(ct, 8 * N, 1));
          okc[ct] = !kHoForceDrop && !kHoDropTarget && (uint32_t)(g >> 32) == tag;
          ok = ok && okc[ct];
          rew[ct] = __uint_as_float((uint32_t)g);
        }
      }
      if (!__builtin_amdgcn_ballot_w64(!ok)) break;
      if (kHoForceDrop || spin >= kHoSpinLimit) {   // the graph's rows are dropped (online side)
        // graphs the target wave has dropped already (its s' wait overran; the LDS flag is stored
        // before its count) are dropped here too but not counted a second time
        bool rest = false;
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
          if (!okc[ct] && *(volatile int*)&TB.tdrop[row0 + min(16 * ct + c, NS - 1)] != 0) {
            okc[ct] = true;
            live_drop[ct] = true;
            nv[ct] = false;
          }
          rest = rest || !okc[ct];
        }
        if (__builtin_amdgcn_ballot_w64(rest)) {
          if (lane == 0) atomicAdd(X.ho_err, 1u);
          drop_overrun<NS, GS>(okc, live_drop, nv, c);
        }
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  if (!online && p == 0) {
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      float qmax = F.q[ct][0];
#pragma unroll
      for (int a = 1; a < kActions; ++a) qmax = fmaxf(qmax, F.q[ct][a]);
      if (16 * ct + c < NS) {
        TB.yq[row0 + 16 * ct + c] = nv[ct] ? A.gamma * qmax : 0.0f;   // y = r + this (online waves)
        if (FUSED) TB.tdrop[row0 + 16 * ct + c] = live_drop[ct] ? 1 : 0;
      }
    }
  }
  if (!online && !waited) __builtin_amdgcn_s_setprio(0);
  if (online && lane == 0) TB.prew[wi] = pre ? 1 : 0;
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
      if (FUSED && TB.tdrop[row0 + nn]) nv[ct] = false;   // the target wave dropped the graph
      float qa = F.q[ct][0];
#pragma unroll
      for (int a = 1; a < kActions; ++a) qa = (act[ct] == a) ? F.q[ct][a] : qa;
      const float delta = nv[ct] ? (qa - (rew[ct] + TB.yq[row0 + nn])) : 0.0f;   // y = r + gamma max Q_tgt(s')
      const float gq = delta * A.grad_scale;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const float4 w = *reinterpret_cast<const float4*>(P + L_W2 + act[ct] * kWRow + 16 * t + 4 * p);
        float wv[4] = {w.x, w.y, w.z, w.w};
        asm volatile("" : "+v"(wv[0]), "+v"(wv[1]), "+v"(wv[2]), "+v"(wv[3]));   // one vector read, not 4 masked ones
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
      if (pre) {   // the pre path's images scaled by this node's gq (rows free since B1)
        float o[2][4];
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) o[t][r] = nv[ct] ? dO1[ct][t][r] * gq : 0.0f;
        if (n < NS) {
          *reinterpret_cast<float4*>(&TB.dO[row0 + n][4 * p]) = make_float4(o[0][0], o[0][1], o[0][2], o[0][3]);
          *reinterpret_cast<float4*>(&TB.dO[row0 + n][16 + 4 * p]) = make_float4(o[1][0], o[1][1], o[1][2], o[1][3]);
          if (conv == SWARM_CONV_GAT) {
#pragma unroll
            for (int ut = 0; ut < CT; ++ut)
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const int u = 16 * ut + 4 * p + r;
                if (u < NS) TB.dp[row0 + n][u] = nv[ct] ? dp1[ct][ut][r] * gq : 0.0f;
              }
          }
        }
        dad1[ct] = nv[ct] ? dad1[ct] * gq : 0.0f;
      }
    }
  }
  __syncthreads();   // B2: dZ / T / R / gq / act / d2 / X / cm of every graph (pre path: dO / dp too)
  SWARM_STAMP(5);
  int np_pre = 0;   // online waves of this block on the pre path
#pragma unroll
  for (int w2 = 0; w2 < GPB; ++w2) np_pre += TB.prew[w2];
  // the parameter products that need only B2's images (each writes its slice of the slab).
  // dW1 = dZ^T T and dW2 = onehot(a) gq R as 16x16x4 MFMA tiles, K = 4 of the block's 32 node
  // rows per step: dW1 tiles (ti, tj) = jobs 2 ti + tj, dW2's 9 action rows in one 16-row tile
  // per column half tj = jobs 4 + tj.  A wave runs three tiles of one column half tj, their
  // chains interleaved with every operand read first (as conditional reads they became a branch
  // and an LDS round trip in front of each MFMA): 24 MFMAs of 32 cycles where the 32x32x2 form
  // had 16 of 64 per product, and dW2 takes 16 rows of work instead of 32.
  auto b2_tiles = [&](int tj) {   // lane (c, p) of the D layout: column c, k-slot / row group p
    float a1[2][8], b1[8], a2[8], b2v[8];
    int an[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int n = 4 * s + p;
      a1[0][s] = TB.dZ[n][c];
      a1[1][s] = TB.dZ[n][16 + c];
      b1[s] = TB.T[n][16 * tj + c];
      b2v[s] = TB.R[n][16 * tj + c];
      an[s] = TB.act[n];
      a2[s] = TB.gq[n];
    }
#pragma unroll
    for (int s = 0; s < 8; ++s) asm volatile("" : "+v"(a2[s]));   // loaded unconditionally
    f32x4 d0 = {0.f, 0.f, 0.f, 0.f}, d1 = {0.f, 0.f, 0.f, 0.f}, d2 = {0.f, 0.f, 0.f, 0.f};
    // the transposed tiles (operands swapped: the same products, the same K order): lane (c, p)
    // holds dW1[out = c (+16)][in = 16 tj + 4p .. 4p + 3] and dW2[action = c][in = ...], four
    // consecutive parameters of one 16-column slab run, stored as ONE 16-B store per tile
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      d0 = mfma16(b1[s], a1[0][s], d0);
      d1 = mfma16(b1[s], a1[1][s], d1);
      d2 = mfma16(b2v[s], an[s] == c ? a2[s] : 0.0f, d2);
    }
    sst4(OFF_W1 + c * kHidden + 16 * tj + 4 * p, d0);
    sst4(OFF_W1 + (16 + c) * kHidden + 16 * tj + 4 * p, d1);
    if (c < kActions) sst4(OFF_W2 + c * kHidden + 16 * tj + 4 * p, d2);
  };
  auto b2_job = [&](int job) {   // the vector sums: job 2 = db1, job 3 = db2 and the loss
    if (job == 2) {
      if (lane < kHidden) {
        float v[kTdRows];
#pragma unroll
        for (int n = 0; n < kTdRows; ++n) v[n] = TB.dZ[n][lane];
        float acc = v[0];
#pragma unroll
        for (int n = 1; n < kTdRows; ++n) acc = acc + v[n];
        sst(OFF_B1 + lane, acc);
      }
    } else if (lane < kActions || lane == 63) {   // db2 / loss: the ordered sum over the 32 rows,
      // 8 rows' reads at a time (each read unconditional: as selects around the reads they became
      // a branch and an LDS round trip per row)
      float acc = 0.0f;
#pragma unroll
      for (int k = 0; k < kTdRows; k += 8) {
        int a8[8];
        float g8[8], d8[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) { a8[j] = TB.act[k + j]; g8[j] = TB.gq[k + j]; d8[j] = TB.d2[k + j]; }
#pragma unroll
        for (int j = 0; j < 8; ++j) asm volatile("" : "+v"(g8[j]), "+v"(d8[j]));
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float v = lane == 63 ? d8[j] : (a8[j] == lane ? g8[j] : 0.0f);
          acc = (k == 0 && j == 0) ? v : acc + v;
        }
      }
      sst(lane == 63 ? N_PARAMS : OFF_B2 + lane, acc);
    }
  };

  const int col = lane & 31, h = lane >> 5;
  if (online) {
    float da_d[CT];
    WSmall<NS>& sm = *V.sm;
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) da_d[ct] = pre ? dad1[ct] : 0.0f;
    if (!pre) {
    // ---- dT^T = W1^T dZ^T on MFMA (the dz registers are the B operand),
    //      dO = dT * (1 - t^2) with the forward's tanh registers
    float dO[CT][2][4];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      const int n = 16 * ct + c;
      // W1 fragments first (16 LDS reads in flight), then the two output tiles' chains interleaved
      float w1f[2][2][4];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int t2 = 0; t2 < 2; ++t2) w1f[t2][t][r] = P[L_W1 + (16 * t + 4 * p + r) * kWRow + 16 * t2 + c];
      f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int t2 = 0; t2 < 2; ++t2) acc[t2] = mfma16(w1f[t2][t][r], dz[ct][t][r], acc[t2]);
#pragma unroll
      for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          dO[ct][t2][r] = nv[ct] ? acc[t2][r] * (1.0f - F.t[ct][t2][r] * F.t[ct][t2][r]) : 0.0f;
      if (n < NS) {
        *reinterpret_cast<float4*>(&TB.dO[row0 + n][4 * p]) = make_float4(dO[ct][0][0], dO[ct][0][1], dO[ct][0][2], dO[ct][0][3]);
        *reinterpret_cast<float4*>(&TB.dO[row0 + n][16 + 4 * p]) = make_float4(dO[ct][1][0], dO[ct][1][1], dO[ct][1][2], dO[ct][1][3]);
      }
    }
    SWARM_STAMP(24);
    // ---- GAT backward (attention part).  g[u][v] = H_u . dO_v on MFMA (A = H rows,
    //      B = the dO registers); lane (c, p) holds g[u = 16 ut + 4 p + r][v = 16 ct + c]
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
    }   // !pre
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
        float dpj[GS];   // read unconditionally (rows of this wave's graph), summed for j < N
#pragma unroll
        for (int j = 0; j < GS; ++j) dpj[j] = TB.dp[row0 + base + j][uu];
#pragma unroll
        for (int j = 0; j < GS; ++j) asm volatile("" : "+v"(dpj[j]));
#pragma unroll
        for (int j = 0; j < GS; ++j) da_s = j < N ? da_s + dpj[j] : da_s;
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
    // ---- target waves: the dW1 / dW2 tiles of column half tj = wi (GPB = 2) or both (GPB = 1);
    //      the vector sums (db1, db2 + loss) too unless the block has pre-path online waves:
    //      theirs is the short side of B2 -> B3 there, and the target waves' products the long one
    for (int tj = wi; tj < 2; tj += GPB) b2_tiles(tj);
    if (np_pre == 0)
      for (int job = 2 + wi; job < 4; job += GPB) b2_job(job);
  }
  if (online && pre) {   // (GPB = 2: one pre wave takes both sums, two split them)
    if (np_pre == 1 || wi == 0) b2_job(2);
    if (np_pre == 1 || wi == 1) b2_job(3);
  }
  SWARM_STAMP(26);   // stamps build: the B2 jobs done, before the B3 wait
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
        // operands read up front and unconditionally (column 8 of X is +0: the padding columns
        // c >= kFeat read it), so no LDS round trip sits between two MFMAs of the chain
        float ha[kTdRows / 4], xb[kTdRows / 4];
#pragma unroll
        for (int ks = 0; ks < kTdRows / 4; ++ks) {
          const int n = 4 * ks + p;
          ha[ks] = TB.dH[n][16 * t + c];
          xb[ks] = TB.X[n][c < kFeat ? c : 8];
        }
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < kTdRows / 4; ++ks) acc = mfma16(ha[ks], xb[ks], acc);
        if (c < kFeat) {
#pragma unroll
          for (int r = 0; r < 4; ++r) sst(OFF_W + (16 * t + 4 * p + r) * kFeat + c, acc[r]);
        }
      } else if (job == 2) {   // att_src (half 0) / att_dst (half 1): sum_n da[n] H[n][col]
        const float* da = h == 0 ? TB.das : TB.dad;
        float v[kTdRows];
#pragma unroll
        for (int n = 0; n < kTdRows; ++n) v[n] = da[n] * TB.H[n][col];
        float acc = v[0];
#pragma unroll
        for (int n = 1; n < kTdRows; ++n) acc = acc + v[n];
        sst((h == 0 ? OFF_ATT_SRC : OFF_ATT_DST) + col, acc);
      } else if (lane < kHidden) {
        float v[kTdRows];
#pragma unroll
        for (int n = 0; n < kTdRows; ++n) v[n] = TB.dO[n][lane];
        float acc = v[0];
#pragma unroll
        for (int n = 1; n < kTdRows; ++n) acc = acc + v[n];
        sst(OFF_BIAS + lane, acc);
      }
    }
  }
  SWARM_STAMP(7);
  SWARM_RTSTAMP(9);
}

}  // namespace swarm
