// swarm_actk.h — body of the acting kernel (reset-free part of the hot path): one wave per
// environment; graph -> GCN.forward -> eps-greedy -> env.step -> replay push.  Shared by
// act_kernel (swarm_act.hip) and the fused training-tick kernel (swarm_tick.hip).
//
// Reference call sites replaced (paths relative to the reference checkout):
//   train_gcn_dqn.py:161-172   graph -> model -> eps-greedy -> env.step -> replay.push
//   simulator.py:59-93         kNN graph -> argmax -> env.step -> metrics
//   go_to_position_scenario.py:83-132, obstacle_avoidance_scenario.py:94-173
#pragma once
#include "swarm_adam.h"
#include "swarm_env.h"
#include "swarm_dl.h"
#include "swarm_gat3.h"

namespace swarm {

enum { MODE_Q = 0, MODE_TICK = 1, MODE_ROLLOUT = 2, MODE_STEP = 3 };

struct ActArgs {
  int B, N, scenario, graph, k, conv, env_offset, flags;
  uint32_t k0, k1;
  float radius;            // SWARM_GRAPH_RADIUS
  int net;                 // swarm_net (fills the padding before params: layout otherwise unchanged)
  const float* params;
  const float* x;          // MODE_Q node features [B*N][7]
  const uint8_t* dense;    // SWARM_GRAPH_DENSE multiplicity
  const int32_t* actions;  // MODE_STEP actions [B][N]
  float* state;            // [B][N][4]
  swarm_replay replay;     // replay.s == nullptr -> no push
  const swarm_ctrl* ctrl;  // MODE_TICK: tick / eps / write_slot
  swarm_act_out out;
  int n_ticks;
  uint32_t tick0;
  float eps;
  int learn;               // MODE_TICK: apply the pending optimizer step first (fused tick)
  swarm_learner lr;
  swarm_adam_cfg hp;
  float* grad_norm_out;    // &ctrl->grad_norm (written by block 0)
  int32_t* sample_out;     // MODE_TICK: this tick's TD batch indices [hp.batch] (or NULL)
  unsigned long long* ho_rec;   // fused tick: [B][ho_stride_granules(N)] hand-off records (swarm_common.h)
};

constexpr int kActWPB = 4;   // waves (= environments) per act block; the block is one Adam workgroup

// One wave per environment in the D layout (swarm_dl.h): lane (c, p) serves agent
// n = 16 ct + c with row group p.  Block-wide work is only the weight image (LDS),
// staged from global memory or produced by the fused Adam prologue.
//
// The first memory round trip's pointers and the geometry lead the parameter list so that
// they arrive preloaded in SGPRs (kernarg preload, -amdgpu-kernarg-preload-count): the
// prologue's loads issue at wave start instead of behind a kernarg-segment fetch.
// SCEN: compile-time scenario (no speculated OA physics).  SPEC fixes graph and conv at
// compile time (SPEC_* in swarm_common.h) — e.g. the headline configuration's kernel
// (complete + GAT) carries no kNN / dense / GCN code; SPEC_RUNTIME reads them from A.
template <int NS>
struct ActSmem {
  WScratch<NS> SW[kActWPB];
  // per wave (<= 8 slots): the tick's pair forces [NS][NS][2], formed from the positions the wave
  // loaded while the prologue's optimizer operands are still in flight (they depend on no weight
  // and no action); 16-slot kernels form them after the argmax in the free H rows instead
  __attribute__((aligned(16))) float FB[kActWPB][NS <= 8 ? 2 * NS * (NS + 1) + 2 * NS + 4 * (NS * NS + NS) : 4];
  __attribute__((aligned(16))) float Pw[N_LDS_PARAMS];
  float red[64];   // the optimizer step's norm (adam_norm2_block)
};

// vb / nvb: this block's index among the nvb acting blocks of the launch (the fused
// training-tick kernel runs acting blocks beside TD blocks).
// HO: fused-tick hand-off publishing (swarm_tick.hip only).  NET: SWARM_NET_GCN (the D-layout
// MFMA forward) or SWARM_NET_GAT3 (swarm_gat3.h; acting only, no learner prologue)
template <int NS, int MODE, int SCEN, int SPEC, bool HO = false, int NET = SWARM_NET_GCN>
__device__ __forceinline__ void act_body(ActSmem<NS>& S, const int vb, const int nvb,
                                         const swarm_ctrl* __restrict__ ctrl, float* state, const float* grad,
                                         const float* w_cur, const float* m_cur, const float* v_cur, int B, int N,
                                         const ActArgs& A) {
  constexpr int CT = DGeom<NS>::CT;
  WScratch<NS>* SW = S.SW;
  float* Pw = S.Pw;
  float* red = S.red;
  SWARM_RTSTAMP(30);
  SWARM_STAMP(0);
#if SWARM_STAMPS == 1   // rollouts, slot 29: where the wave runs (HW_ID in the low word, XCC_ID in the high word)
  if (MODE == MODE_ROLLOUT && g_swarm_stamps && (threadIdx.x & 63) == 0)
    g_swarm_stamps[((size_t)blockIdx.x * 16 + (threadIdx.x >> 6)) * 32 + 29] =
        (unsigned long long)__builtin_amdgcn_s_getreg(4 | (31 << 11)) |
        ((unsigned long long)__builtin_amdgcn_s_getreg(20 | (15 << 11)) << 32);
#endif
  if (HO) __builtin_amdgcn_s_setprio(3);   // fused tick: acting waves ahead of the TD blocks beside them
  const int w = threadIdx.x >> 6;
  const DGeom<NS> d = make_dgeom<NS>(vb * kActWPB + w, B);
  const int graph = spec_graph<SPEC>(A.graph);
  const int conv = spec_conv<SPEC>(A.conv);
  // the kNN tie memo pays only across the ticks of one launch: rollouts
  WView<NS> V = SW[w].view();
  if constexpr (MODE == MODE_ROLLOUT) {
    SW[w].memo.clear(threadIdx.x & 63);
    wave_lds_sync();
  } else {
    V.memo = nullptr;
  }
  WSmall<NS>& sm = SW[w].sm;
  const int c = d.c, p = d.p;

  // prologue: every independent global load in flight at once.  The fused tick always learns
  // (HO), so its optimizer-step operands are loaded first, from the preloaded pointers, ahead
  // of anything that waits on ctrl or the kernarg segment
  constexpr bool kLearnCT = MODE == MODE_TICK && NET == SWARM_NET_GCN && HO;
  DFwd<NS> F;
  float px[CT], py[CT], vx[CT], vy[CT];
  bool valid[CT];
  size_t node[CT];
  // the state first: the pair forces below need only it, and run while the optimizer operands
  // (issued right after) are in flight
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    const int n = 16 * ct + c;
    valid[ct] = d.live && n < N;
    node[ct] = (size_t)d.gid * N + min(n, N - 1);   // idle lanes alias an in-bounds node, never store
    px[ct] = py[ct] = vx[ct] = vy[ct] = 0.0f;
    if (MODE == MODE_Q) {
      F.x[ct][0] = valid[ct] ? A.x[node[ct] * kFeat + p] : 0.0f;
      F.x[ct][1] = (valid[ct] && 4 + p < kFeat) ? A.x[node[ct] * kFeat + 4 + p] : 0.0f;
    } else {
      const float4 st = *reinterpret_cast<const float4*>(state + node[ct] * 4);
      if (valid[ct]) { px[ct] = st.x; py[ct] = st.y; vx[ct] = st.z; vy[ct] = st.w; }
    }
  }
  AdamRegs R;
  if (kLearnCT) R.load(grad, w_cur, m_cur, v_cur, threadIdx.x, true);
  // Flocking: the scenario's per-agent previous_distance_to_agents (flocking_scenario.py:110-122,
  // 163-164), kept after the [B][N][4] state as [B][N] floats (swarm_hip.h, swarm_env_reset)
  float* fl_prev = (SCEN == SWARM_FLOCKING && MODE != MODE_Q) ? state + (size_t)B * N * 4 : nullptr;
  float spread[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) spread[ct] = (fl_prev && valid[ct] && p == 0) ? fl_prev[node[ct]] : 0.0f;
  // the whole control block in registers, loaded once and up front (two scalar lines in
  // flight together instead of dependent loads behind branches)
  swarm_ctrl cc = {};
  if (MODE == MODE_TICK) cc = *ctrl;
  uint32_t tick = A.tick0;
  float eps = A.eps;
  uint32_t slot = 0;
  if (MODE == MODE_TICK) {
    tick = cc.tick;
    eps = cc.eps;
    slot = cc.write_slot;
  }
  const uint32_t genv = (uint32_t)(A.env_offset + d.gid);
  // the first tick's eps-greedy coin only needs ctrl: drawn while the prologue's loads fly
  const bool explore0 = (MODE != MODE_STEP && MODE != MODE_Q && eps > 0.0f) &&
                        u01(philox4x32(tick, genv, STREAM_COIN, 0u, A.k0, A.k1).x) < eps;
  // fused tick: is this env's transition in the TD batch drawn from this tick's slot?
  // (position of graph id slot * B + env in the keyed permutation < batch)
  bool ho_pub = false;
  if (MODE == MODE_TICK && HO && d.live) {
    const uint32_t cap = (uint32_t)A.replay.capacity;
    const uint32_t filled = cc.filled_slots;
    const uint32_t ng = (filled + 1 < cap ? filled + 1 : cap) * (uint32_t)B;
    if (ng >= (uint32_t)A.hp.batch) {
      const SampleKey sk = sample_key_cached(&cc, ng, A.k0 ^ ((uint32_t)A.env_offset * 0x9E3779B9u), A.k1, tick);
      ho_pub = sample_position(slot * (uint32_t)B + (uint32_t)d.gid, sk) < (uint32_t)A.hp.batch;
    }
  }
  // the late stores' pointers, fetched from the kernarg segment beside the wait explore0
  // already has
  float* rp_s = A.replay.s;
  float* rp_sn = A.replay.s_next;
  float* rp_r = A.replay.r;
  uint8_t* rp_a = A.replay.a;
  float* o_rew = A.out.reward;
  float* o_avg = A.out.avg_dist;
  float* o_hits = A.out.hits;
  int32_t* smp = A.sample_out;
  // fused tick: s of a sampled transition is the state loaded above, so it is published now, a
  // whole optimizer step and forward ahead of a: the waiting online TD wave runs its forward on
  // s (and its gq-free backward once a lands) while this wave computes (swarm_tdk.h, pre path)
  unsigned long long* ho_r = nullptr;
  const uint32_t ho_tag = cc.tick + 1u;
  if (MODE == MODE_TICK && HO && ho_pub) {
    ho_r = A.ho_rec + (size_t)d.gid * ho_stride_granules(N);
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
      if (valid[ct])
        st_granule(ho_r + 4 * (16 * ct + c) + p, ho_tag,
                   __float_as_uint(p == 0 ? px[ct] : (p == 1 ? py[ct] : (p == 2 ? vx[ct] : vy[ct]))));
  }
  // ---- VMAS pair forces of this tick's positions (World._get_constraint_forces): they need no
  //      weight and no action, so the first tick's are formed here, while the optimizer operands
  //      are in flight, instead of between the argmax and the integrator.  64 / NS lanes per agent
  //      (NS = 8: one pair per lane), each pair into FB[n][u]; the force sum after the argmax adds
  //      them in VMAS order.  -f(p_u - p_v) == f(p_v - p_u) bit for bit.
  constexpr bool kHoist = NS <= 8 && NET == SWARM_NET_GCN;
  // pair-force scratch: FB (hoisted), else the H / T / R rows, free after the forward
  float* fb = kHoist ? S.FB[w] : &SW[w].H[0][0];
  // row n of the force matrix at a stride of NS + 1 float2: the force sum's 16 lanes (one agent
  // each) read 16 distinct LDS banks instead of 2 (a stride of 2 NS floats is a multiple of 32)
  constexpr int kFbRow = 2 * (NS + 1);
  // then the obstacle pair of every agent (OA) and the list of the tick's pairs in contact
  constexpr int kFbOb = NS * kFbRow;
  constexpr int kFbList = kFbOb + 2 * NS;      // [NS * NS + NS][4]: dx, dy, dist, destination
  // Only where a lane has more than one candidate (16 slots: 4 pair slots; OA: + the obstacle).
  // GoTo with 8 slots (one pair per lane) and 32 slots (no room for the list) evaluate each pair
  // in place, as pair_force does: the list only costs there (C2 13.72 -> 13.76 us per tick)
  constexpr bool kCompact = NS <= 16 && (NS * NS / 64 + (SCEN == SWARM_OBSTACLE_AVOIDANCE ? 1 : 0)) > 1;
  static_assert(3 * NS * kRow >= (kCompact ? kFbList + 4 * (NS * NS + NS) : kFbOb + 2 * NS), "pair-force scratch");
  // Every pair's distance and contact test first; pairs out of contact get exactly 0 (the
  // reference's torch.where); the pairs in contact (and agents touching the obstacle) are then
  // compacted into a list and evaluated 64 at a time, one per lane, so the transcendental part
  // runs once per 64 contacts instead of once per pair slot that any lane has in contact (with 16
  // slots: 4 pair slots + the obstacle per lane).  Same operations per pair as pair_force.
  auto pair_forces = [&]() {
    if (kHoist || MODE == MODE_STEP) {   // else the forward left the positions in sm.px / sm.py
#pragma unroll
      for (int ct = 0; ct < CT; ++ct)
        if (16 * ct + c < NS && p == 0) { sm.px[16 * ct + c] = px[ct]; sm.py[16 * ct + c] = py[ct]; }
      wave_lds_sync();
    }
    constexpr int LPN = 64 / NS, NPL = NS / LPN;
    const int n = d.lane / LPN;
    const float pxn = sm.px[n], pyn = sm.py[n];
    float cdx[NPL + 1], cdy[NPL + 1], cds[NPL + 1];
    int cof[NPL + 1];
    bool cin[NPL + 1];
#pragma unroll
    for (int j = 0; j < NPL; ++j) {
      const int u = d.lane % LPN + LPN * j;
      cdx[j] = pxn - sm.px[u];
      cdy[j] = pyn - sm.py[u];
      cds[j] = norm2(cdx[j], cdy[j]);
      cin[j] = u < N && n < N && pair_contact(cds[j]);   // u == n: distance 0, no contact
      cof[j] = n * kFbRow + 2 * u;
      float2 g = make_float2(0.0f, 0.0f);
      if (!kCompact && cin[j]) contact_force(cdx[j], cdy[j], cds[j], g.x, g.y);
      if (!kCompact || !cin[j]) *reinterpret_cast<float2*>(fb + cof[j]) = g;
    }
    {   // the obstacle pair of agent n, on the agent's first lane
      const bool lead = d.lane % LPN == 0;
      cdx[NPL] = pxn - kObstX;
      cdy[NPL] = pyn - kObstY;
      cds[NPL] = norm2(cdx[NPL], cdy[NPL]);
      cin[NPL] = SCEN == SWARM_OBSTACLE_AVOIDANCE && lead && n < N && pair_contact(cds[NPL]);
      cof[NPL] = kFbOb + 2 * n;
      float2 g = make_float2(0.0f, 0.0f);
      if (!kCompact && cin[NPL]) contact_force(cdx[NPL], cdy[NPL], cds[NPL], g.x, g.y);
      if (SCEN == SWARM_OBSTACLE_AVOIDANCE && lead && (!kCompact || !cin[NPL])) *reinterpret_cast<float2*>(fb + cof[NPL]) = g;
    }
    if constexpr (!kCompact) return;
    uint32_t total = 0;
#pragma unroll
    for (int j = 0; j <= NPL; ++j) {
      const unsigned long long m = __builtin_amdgcn_ballot_w64(cin[j]);
      if (cin[j]) {
        const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        *reinterpret_cast<float4*>(fb + kFbList + 4 * (total + below)) =
            make_float4(cdx[j], cdy[j], cds[j], __int_as_float(cof[j]));
      }
      total += (uint32_t)__builtin_popcountll(m);
    }
    if (total != 0u) {
      wave_lds_sync();
      for (uint32_t k0 = 0; k0 < total; k0 += 64) {
        const uint32_t k = k0 + (uint32_t)d.lane;
        if (k < total) {
          const float4 e = *reinterpret_cast<const float4*>(fb + kFbList + 4 * k);
          float gx, gy;
          contact_force(e.x, e.y, e.z, gx, gy);
          *reinterpret_cast<float2*>(fb + __float_as_int(e.w)) = make_float2(gx, gy);
        }
      }
    }
  };
  // hoisted for graphs of <= 8 agents (one pair per lane); with 16 slots (4 pairs per lane) the
  // same hoist measured slower at C3 (18.17 -> 18.82 us per tick, 66 instead of 45 SGPR spills:
  // profiles/r05_ab_hoist_forces_c3.jsonl), so there the forces keep their place after the argmax
  if (MODE != MODE_Q && kHoist) pair_forces();
  // ...and the first tick's random actions of an exploring env (train_gcn_dqn.py:164-165)
  int ract0[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    ract0[ct] = 0;
    if (kHoist && explore0) {
      const int agent = min(16 * ct + c, N - 1);
      const u32x4 wd = philox4x32(tick, genv, STREAM_RAND_ACTION, (uint32_t)(agent >> 2), A.k0, A.k1);
      const int j = agent & 3;
      ract0[ct] = uniform_int(j == 0 ? wd.x : (j == 1 ? wd.y : (j == 2 ? wd.z : wd.w)), kActions);
    }
  }
  if (MODE == MODE_TICK && NET == SWARM_NET_GCN && (kLearnCT || A.learn)) {
    // fused optimizer step of the previous tick's TD gradient (train_gcn_dqn.py:125-133)
    static_assert(64 * kActWPB == kAdamNT, "the act block is one Adam workgroup");
    const int tid = threadIdx.x;
    if (!kLearnCT) R.load(grad, w_cur, m_cur, v_cur, tid, true);
    const uint32_t pending = cc.peer_hold ? 0u : cc.trained;   // a held rank applies no step
    const uint32_t tnow = cc.tick;
    const float step_size = cc.adam_step_size, inv_bc2 = cc.adam_inv_bc2;
    float gn = 0.0f;
    SWARM_STAMP(20);
    if (pending)
      gn = adam_apply<21>(R, A.hp, step_size, inv_bc2, cc.one_m_beta1, cc.one_m_beta2, tid, red,
                          (A.hp.flags & SWARM_ADAM_F_NORM_PARTIALS) != 0);
    store_w_lds(Pw, R, tid);
    SWARM_STAMP(24);
    if (vb == 0) {
      store4(A.lr.w_nxt, R.w, R.wt, tid);
      store4(A.lr.m_nxt, R.m, R.mt, tid);
      store4(A.lr.v_nxt, R.v, R.vt, tid);
      if (pending && (tnow % (uint32_t)A.hp.update_target_every) == 0u) store4(A.lr.target, R.w, R.wt, tid);
      if (pending && tid == 0 && A.grad_norm_out) *A.grad_norm_out = gn;
    }
  } else if (MODE != MODE_STEP && NET == SWARM_NET_GAT3) {
    for (int i = threadIdx.x; i < G3_N_PARAMS; i += 64 * kActWPB) Pw[i] = A.params[i];
  } else if (MODE != MODE_STEP) {
    ParamStage<64 * kActWPB> ps;
    ps.load(A.params, threadIdx.x);
    ps.store(Pw, threadIdx.x);
  }
  __syncthreads();   // weight image complete
  const float* P = Pw;
  SWARM_STAMP(1);

  const int n_ticks = (MODE == MODE_ROLLOUT) ? A.n_ticks : 1;
  float rew_sum[CT], hits_sum = 0.0f;
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) rew_sum[ct] = 0.0f;

  for (int it = 0; it < n_ticks; ++it) {
#if SWARM_STAMPS == 1   // stamps build: the wave's slowest tick (slot 25 cycles, slot 19 tick index)
    const long long t_tick0 = clock64();
#endif
    if (MODE != MODE_Q && kHoist && it > 0) pair_forces();   // this tick's positions
    if (MODE != MODE_Q) {
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        node_x(px[ct], py[ct], vx[ct], vy[ct], 16 * ct + c, p, F.x[ct]);
        if (!valid[ct]) { F.x[ct][0] = 0.0f; F.x[ct][1] = 0.0f; }
      }
    }
    if (MODE != MODE_STEP && NET == SWARM_NET_GAT3) {
      gat3_forward<NS>(P, d, N, graph, A.k, A.radius, A.dense, V, F);
    } else if (MODE != MODE_STEP) {
      dl_forward<NS, 8>(P, d, N, graph, A.k, A.radius, conv, A.dense, V, false, F);
    }
    if (it == 0) SWARM_STAMP(2);

    if (MODE == MODE_Q) {   // the node's row groups store its Q row (from LDS: no lane-indexed registers)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct)
        if (valid[ct])
          for (int a = p; a < kActions; a += 4) A.out.q[node[ct] * kActions + a] = sm.Q[16 * ct + c][a];
      return;
    }

    // ---- eps-greedy (train_gcn_dqn.py:164-167), one Philox coin per env and tick
    const uint32_t tk = tick + (uint32_t)it;
    bool explore = explore0;
    if (it > 0 && eps > 0.0f) explore = u01(philox4x32(tk, genv, STREAM_COIN, 0u, A.k0, A.k1).x) < eps;
    int action[CT];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      const int agent = min(16 * ct + c, N - 1);
      action[ct] = (MODE == MODE_STEP) ? (valid[ct] ? A.actions[node[ct]] : 0) : argmax9(F.q[ct]);
      if (explore) {   // the action draw only runs on exploring envs (the first tick's: drawn above)
        if (kHoist && it == 0) {
          action[ct] = ract0[ct];
        } else {
          const u32x4 wd = philox4x32(tk, genv, STREAM_RAND_ACTION, (uint32_t)(agent >> 2), A.k0, A.k1);
          const int j = agent & 3;
          const uint32_t word = j == 0 ? wd.x : (j == 1 ? wd.y : (j == 2 ? wd.z : wd.w));
          action[ct] = uniform_int(word, kActions);
        }
      }
    }

    // fused tick: this env's transition is in the tick's TD batch -> publish it as tagged
    // write-through granules as soon as each part exists (swarm_common.h hand-off record):
    // s at the prologue (above), a now (the online TD wave's gq-free backward), s' after the
    // integrator (the target TD wave's forward input), r after the reward (needed only for y)
    if (MODE == MODE_TICK && HO && ho_r) {
#pragma unroll
      for (int ct = 0; ct < CT; ++ct)
        if (valid[ct] && p == 3) st_granule(ho_r + 9 * N + 16 * ct + c, ho_tag, (uint32_t)action[ct]);
    }
    if (it == 0) SWARM_STAMP(5);
    // ---- env.step (VMAS World.step + scenario reward).  The 4 row groups of an agent
    //      split its partner pairs (group p: partners p, p + 4, ...), then every lane sums
    //      the forces in VMAS order: 0 + u, obstacle pair, agent pairs in ascending partner
    //      index; -f(p_u - p_v) == f(p_v - p_u) bit for bit.
    if (MODE != MODE_Q && !kHoist) pair_forces();   // (16 slots: here, after the argmax)
    if (it == 0) SWARM_STAMP(6);
    wave_lds_sync();
    if (it == 0) SWARM_STAMP(7);
    StepOut o[CT];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      const int n = min(16 * ct + c, NS - 1);
      float fx = 0.0f + action_level(action[ct] / 3);
      float fy = 0.0f + action_level(action[ct] % 3);
      if (SCEN == SWARM_OBSTACLE_AVOIDANCE) {   // the obstacle pair (pair_forces)
        const float2 g = *reinterpret_cast<const float2*>(fb + kFbOb + 2 * n);
        fx = fx + g.x; fy = fy + g.y;
      }
      // every slot read at once, no per-partner branch: slots u >= N hold +0 and fx, fy
      // (started from +0 or +-1) never become -0, so adding them is exact
      float2 f[NS];
#pragma unroll
      for (int u = 0; u < NS; ++u) f[u] = *reinterpret_cast<const float2*>(fb + n * kFbRow + 2 * u);
#pragma unroll
      for (int u = 0; u < NS; ++u) { fx = fx + f[u].x; fy = fy + f[u].y; }
      o[ct] = integrate(px[ct], py[ct], vx[ct], vy[ct], fx, fy);
      if (MODE == MODE_TICK && HO && ho_r && valid[ct]) {
        const int nn = 16 * ct + c;
        const float v = p == 0 ? o[ct].px : (p == 1 ? o[ct].py : (p == 2 ? o[ct].vx : o[ct].vy));
        st_granule(ho_r + 4 * N + 4 * nn + p, ho_tag, __float_as_uint(v));
      }
      if (16 * ct + c < NS && p == 0) {
        if (SCEN == SWARM_FLOCKING) { sm.aux[16 * ct + c] = o[ct].px; sm.aux2[16 * ct + c] = o[ct].py; }
        else { sm.aux[16 * ct + c] = o[ct].dgoal; sm.aux2[16 * ct + c] = (o[ct].dobs <= 0.2f) ? 1.0f : 0.0f; }
      }
    }
    if (it == 0) SWARM_STAMP(3);
    if (MODE == MODE_TICK && HO && ho_r) SWARM_RTSTAMP(29);   // s' published (stamps build only)
    wave_lds_sync();
    float rf = 0.0f;   // flocking: the collective reward
    if (SCEN == SWARM_FLOCKING) {
      // every agent's term from its post-step distances (sm.aux/aux2) and the scenario's stored
      // values: the goal term's equals the pre-step distance (set at reset from the new
      // position, flocking_scenario.py:102-107, then by every reward call :140-142); the
      // spread's is carried in `spread` (reset loop value after a reset, :110-122; :163-164)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        const int n = 16 * ct + c;
        if (n < NS && p == 0) {
          const float dpre = norm2(px[ct] - kGoalX, py[ct] - kGoalY);
          float spost = 0.0f, cnt = 0.0f;
          for (int j = 0; j < N; ++j) {
            if (j == n) continue;
            const float bn = norm2(o[ct].px - sm.aux[j], o[ct].py - sm.aux2[j]);
            const float b = bn - kFlockDesired;
            spost = spost + b * b;
            if ((bn - kRadius) - kRadius <= kFlockContact) cnt = cnt + 1.0f;   // World.get_distance
          }
          const float others = (float)(N - 1);   // torch mean over the N - 1 other agents
          const float d_pre = spread[ct], d_post = (spost / others) * kFlockShaping;
          spread[ct] = d_post;
          float rg = dpre * kFlockShaping - o[ct].dgoal * kFlockShaping;               // :140-141
          if (o[ct].dgoal < kRadius) rg = rg + kFlockGoalBonus;                      // on_goal :138, 146-147
          const float term = (rg + (-cnt)) + (d_pre - d_post);                       // :128-129
          fb[n] = (n < N) ? term : 0.0f;
          fb[NS + n] = cnt;
          fb[2 * NS + n] = o[ct].dgoal;
        }
      }
      wave_lds_sync();
      rf = fb[0];
#pragma unroll
      for (int j = 1; j < NS; ++j)
        if (j < N) rf = rf + fb[j];
    }
    float dj[NS], hj[NS];
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      if (SCEN == SWARM_FLOCKING) { dj[j] = fb[2 * NS + (j < N ? j : 0)]; hj[j] = fb[NS + (j < N ? j : 0)]; }
      else { dj[j] = sm.aux[j < N ? j : 0]; hj[j] = sm.aux2[j < N ? j : 0]; }
    }
    float dsum = dj[0], hsum = hj[0];
#pragma unroll
    for (int j = 1; j < NS; ++j)
      if (j < N) { dsum = dsum + dj[j]; hsum = hsum + hj[j]; }
    float rg = 0.0f;
    if (SCEN == SWARM_GOTO) {
      rg = -dj[0];
#pragma unroll
      for (int j = 1; j < NS; ++j)
        if (j < N) rg = rg + (-dj[j]);   // go_to_position_scenario.py:112-113
    }
    if (it == 0) SWARM_STAMP(13);
    const float avg = dsum / (float)N;
    if (SCEN == SWARM_GOTO) hsum = 0.0f;

#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      const float rew = (SCEN == SWARM_GOTO) ? rg : (SCEN == SWARM_FLOCKING ? rf : oa_reward(o[ct].dgoal, o[ct].dobs));
      if (MODE == MODE_TICK && HO && ho_r && valid[ct] && p == 0)
        st_granule(ho_r + 8 * N + 16 * ct + c, ho_tag, __float_as_uint(rew));
      const int n = 16 * ct + c;
      if (valid[ct]) {   // the node's four row groups share its stores
        if (MODE == MODE_TICK || MODE == MODE_STEP) {
          if (MODE == MODE_TICK && A.out.q)
            for (int a = p; a < kActions; a += 4) A.out.q[node[ct] * kActions + a] = sm.Q[n][a];
          if (MODE == MODE_TICK && A.out.mult && graph != SWARM_GRAPH_DENSE)
            for (int u = p; u < N; u += 4)
              A.out.mult[((size_t)d.gid * N + u) * N + n] = (uint8_t)in_mult<NS>(u, n, N, graph, sm, nullptr, d.gid);
          if (p == 0) {
            if (A.out.actions) A.out.actions[node[ct]] = action[ct];
            if (o_rew) o_rew[node[ct]] = rew;
            if (n == 0) {
              if (o_avg) o_avg[d.gid] = avg;
              if (o_hits) o_hits[d.gid] = hsum;
            }
          } else if (MODE == MODE_TICK && rp_s) {
            const size_t ri = ((size_t)slot * B + d.gid) * N + n;
            if (p == 1) reinterpret_cast<float4*>(rp_s)[ri] = make_float4(px[ct], py[ct], vx[ct], vy[ct]);
            else if (p == 2) reinterpret_cast<float4*>(rp_sn)[ri] = make_float4(o[ct].px, o[ct].py, o[ct].vx, o[ct].vy);
            else { rp_r[ri] = rew; rp_a[ri] = (uint8_t)action[ct]; }
          }
          if (p == 3 && A.out.obs) {
            float* ob = A.out.obs + node[ct] * 6;
            ob[0] = o[ct].px; ob[1] = o[ct].py; ob[2] = o[ct].vx; ob[3] = o[ct].vy; ob[4] = kGoalX; ob[5] = kGoalY;
          }
        } else if (p == 0) {  // MODE_ROLLOUT
          if (A.out.traj_pos) {
            const size_t ti = ((size_t)it * B + d.gid) * N + n;
            reinterpret_cast<float2*>(A.out.traj_pos)[ti] = make_float2(o[ct].px, o[ct].py);
          }
          if (n == 0) {
            if (A.out.traj_dist) A.out.traj_dist[(size_t)it * B + d.gid] = avg;
            if (A.out.traj_hits) A.out.traj_hits[(size_t)it * B + d.gid] = hsum;
          }
        }
      }
      rew_sum[ct] = rew_sum[ct] + rew;
      px[ct] = o[ct].px; py[ct] = o[ct].py; vx[ct] = o[ct].vx; vy[ct] = o[ct].vy;
    }
    hits_sum = hits_sum + hsum;
    if (it == 0) SWARM_STAMP(14);
    if (MODE == MODE_ROLLOUT && it == n_ticks - 1 && c == 0 && p == 0 && d.live) {
      if (A.out.avg_dist) A.out.avg_dist[d.gid] = avg;
      if (A.out.hits) A.out.hits[d.gid] = hits_sum;
    }
    wave_lds_sync();   // every lane done with this tick's LDS rows before the next tick rewrites them
#if SWARM_STAMPS == 1
    if (g_swarm_stamps && (threadIdx.x & 63) == 0) {
      unsigned long long* ws = g_swarm_stamps + ((size_t)blockIdx.x * 16 + (threadIdx.x >> 6)) * 32;
      const unsigned long long dt = (unsigned long long)(clock64() - t_tick0);
      if (dt > ws[25]) { ws[25] = dt; ws[19] = (unsigned long long)it; }
    }
#endif
  }
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    if (valid[ct] && p == 0) {
      reinterpret_cast<float4*>(state)[node[ct]] = make_float4(px[ct], py[ct], vx[ct], vy[ct]);
      if (fl_prev) fl_prev[node[ct]] = spread[ct];
      if (MODE == MODE_ROLLOUT) {
        if (A.out.reward) A.out.reward[node[ct]] = rew_sum[ct];
        if (A.out.obs) {
          float* ob = A.out.obs + node[ct] * 6;
          ob[0] = px[ct]; ob[1] = py[ct]; ob[2] = vx[ct]; ob[3] = vy[ct]; ob[4] = kGoalX; ob[5] = kGoalY;
        }
      }
    }
  }
if (MODE == MODE_TICK && smp) {   // at the end of every wave: nothing waits on it
    // this tick's TD batch (GraphReplayBuffer.sample, train_gcn_dqn.py:40): the keyed
    // permutation of swarm_td_grad's in-kernel draw, one index per lane of a wave; the
    // key comes from ctrl's cache (prepared by the previous reduce launch)
    const uint32_t cap = (uint32_t)A.replay.capacity;
    const uint32_t filled = cc.filled_slots;
    const uint32_t ng = (filled + 1 < cap ? filled + 1 : cap) * (uint32_t)B;
    if (ng >= (uint32_t)A.hp.batch) {
      const SampleKey sk = sample_key_cached(&cc, ng, A.k0 ^ ((uint32_t)A.env_offset * 0x9E3779B9u), A.k1, tick);
      const int nw = nvb * kActWPB;
      for (int i = vb * kActWPB + w + nw * d.lane; i < A.hp.batch; i += nw * 64)
        smp[i] = (int32_t)sample_index((uint32_t)i, sk);
    }
  }
  SWARM_STAMP(4);
  SWARM_RTSTAMP(31);
}

}  // namespace swarm
