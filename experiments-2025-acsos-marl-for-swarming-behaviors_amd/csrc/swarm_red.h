// swarm_red.h — the slab reduce's tick-advance pieces, shared by the reduce launch
// (grad_reduce_kernel, swarm_td.hip) and the one-launch tick (swarm_tick.hip with
// SWARM_F_TICK_REDUCE), where acting blocks take the reduce's roles once their env is stepped.
//
// One launch per tick: a kernel boundary costs ≈1.9 µs of the tick in a hipGraph chain (an
// empty kernel's period, bench.py kernel_us.ctrl_advance_kernel), about the reduce launch's
// whole share.  Inside the tick kernel:
//  - TD blocks store their slab as tagged granules {tag = tick + 1, value} with write-through
//    stores (swarm_common.h st_granule) and count themselves done (td_done);
//  - acting blocks count themselves past their prologue (act_pro: ctrl, grad, w/m/v read);
//  - acting blocks 1..105 are the column roles: once every acting block has read grad
//    (act_pro) and most TD blocks are done, they sweep their 16 columns' granules until every
//    tag is this tick's (the data is its own flag, no fence), then sum in the reduce launch's
//    exact order (64 groups of consecutive slabs, 8 runs of 8, the run sums) and write grad;
//  - acting block 106 is the control role (the reduce launch's control block, red_control)
//    and advances the workspace's epoch, so the next launch's counts start afresh;
//  - acting block 0 copies w / m / v _nxt -> _cur: it wrote _nxt itself, so its own loads see
//    them without a fence.
// Control and copy wait until every block has read ctrl and _cur (act_pro, td_done).  Every
// wait is bounded (kHoSpinLimit) and counted in the workspace's error word.
#pragma once
#include "swarm_actk.h"
#include "swarm_tdk.h"

namespace swarm {

constexpr int kRedCols = 16;      // columns per reduce block
constexpr int kRedGroups = 64;    // slab groups per column (consecutive slabs each)
constexpr int kRedRuns = kRedGroups / 8;
constexpr int kRedChunk = 8;      // slabs per load chunk of a group
constexpr int kRedColBlocks = (N_PARAMS + 1 + kRedCols - 1) / kRedCols;

// ---- the ctrl advance of one tick (the reduce launch's control block).  Every thread of the
//      block calls it; thread 0 advances the counters and the Adam scalars, thread 64 derives the
//      next tick's sampling key; both read ctrl before the barrier and write after it.
struct RedCtrl {
  int capacity, B, batch;
  swarm_adam_cfg hp;
  uint32_t k0, k1;   // replay-sampling key (seed ^ rank salt)
};

__device__ inline void red_control(swarm_ctrl* C, const RedCtrl& A) {
  const int t = threadIdx.x;
  uint32_t c_trained = 0, c_step = 0, c_tick = 0, c_slot = 0, c_filled = 0;
  double b1p = 1.0, b2p = 1.0;
  float next_step_size = 0.0f, next_inv_bc2 = 0.0f;
  SampleKey nk = {};
  uint32_t nk_n = 0, nk_tick = 0;
  const uint32_t cap = (uint32_t)A.capacity;
  if (t == 0) {
    // a held rank (peer_hold: an expired exchange wait) applied no step this tick
    c_trained = C->peer_hold ? 0u : C->trained;
    c_step = C->adam_step; c_tick = C->tick; c_slot = C->write_slot; c_filled = C->filled_slots;
    b1p = ctrl_get_double(C, CTRL_B1POW);
    b2p = ctrl_get_double(C, CTRL_B2POW);
    if (c_trained) {   // the step this tick's act kernel applied
      b1p = b1p * (double)A.hp.beta1;
      b2p = b2p * (double)A.hp.beta2;
      adam_next_scalars(A.hp, b1p, b2p, next_step_size, next_inv_bc2);
    }
  } else if (t == 64) {
    const uint32_t filled = C->filled_slots;
    const uint32_t f1 = filled + 1 < cap ? filled + 1 : cap;   // filled after this tick
    nk_n = (f1 + 1 < cap ? f1 + 1 : cap) * (uint32_t)A.B;       // graphs the next tick samples from
    nk_tick = C->tick + 1;
    nk = sample_key(nk_n, A.k0, A.k1, nk_tick);
  }
  __syncthreads();
  if (t == 0) {   // record the pending update, advance the tick
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
    C->tick = c_tick + 1;
    C->write_slot = (c_slot + 1) % cap;
    C->filled_slots = valid_slots;
  } else if (t == 64) {
    C->sample_key[0] = nk.rk[0]; C->sample_key[1] = nk.rk[1]; C->sample_key[2] = nk.rk[2]; C->sample_key[3] = nk.rk[3];
    C->sample_bits = (uint32_t)nk.bits;
    C->sample_n = nk_n;
    C->sample_tick = nk_tick;
  }
}

// ---- one-launch tick (SWARM_F_TICK_REDUCE)
// counters: the workspace's 64-bit words kWsActPro (acting blocks past their prologue) and
// kWsTdDone (TD blocks whose slab granules are issued), {epoch << 16 | count}; the control role
// advances kWsEpoch (swarm_common.h)
constexpr int kRedRoleCopy = 0;                        // acting block 0: w / m / v _nxt -> _cur
constexpr int kRedRoleCol0 = 1;                        // acting blocks 1 .. 105: column blocks
constexpr int kRedRoleCtrl = kRedRoleCol0 + kRedColBlocks;   // acting block 106: ctrl advance
constexpr int kRedRoles = kRedRoleCtrl + 1;            // acting blocks a one-launch tick needs
constexpr int kRedMaxPer = 8;                          // slabs per group: n_slabs <= 512
#ifndef SWARM_RED_LEAD
#define SWARM_RED_LEAD 16   // column roles start sweeping when all but this many TD blocks are done
#endif
#ifndef SWARM_RED_SLEEP
#define SWARM_RED_SLEEP 4   // s_sleep argument (x 64 cycles) between two sweeps / polls
#endif

struct RedTick {
  unsigned long long* ws;            // the tick workspace (error word, counters, epoch)
  uint32_t* err;                     // the workspace's error word
  const unsigned long long* slabs;   // tagged slab granules (slab_index layout)
  int n_slabs, n_act;
  float* grad;
  swarm_learner lr;
  int N;
  RedCtrl ctl;
};

struct RedSmem {
  float part[kRedGroups][kRedCols];
  float part2[kRedRuns][kRedCols];
};

// bounded wait until this epoch's count in *w reaches want: thread 0 polls (one request per
// poll, not one per lane of every waiting wave: hundreds of waves hammering one line starve the
// very atomics they wait for), the block waits at the barrier
__device__ inline void red_wait(const unsigned long long* w, unsigned long long epoch, uint32_t want, uint32_t* err) {
  if (threadIdx.x == 0) {
    for (int spin = 0;; ++spin) {
      const unsigned long long v = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((v >> 16) == epoch && (uint32_t)(v & 0xFFFFull) >= want) break;
      if (spin >= kHoSpinLimit) {
        atomicAdd(err, 1u);
        break;
      }
      __builtin_amdgcn_s_sleep(SWARM_RED_SLEEP);
    }
  }
  __syncthreads();
}

// the acting block's reduce role (vb < kRedRoles), 256 threads; tick / epoch as read at launch
__device__ inline void red_role(int vb, const RedTick& R, swarm_ctrl* C, uint32_t tick, unsigned long long epoch,
                                RedSmem& L) {
  __syncthreads();   // the block's LDS (the acting union member) is free from here
  SWARM_RTSTAMP(15);
  const uint32_t n_td = (uint32_t)R.n_slabs;
  red_wait(R.ws + kWsActPro, epoch, (uint32_t)R.n_act, R.err);   // every acting block read grad / ctrl / _cur
  SWARM_RTSTAMP(16);
  if (vb == kRedRoleCopy || vb == kRedRoleCtrl) {
    red_wait(R.ws + kWsTdDone, epoch, n_td, R.err);   // every TD block read ctrl / _cur
    if (vb == kRedRoleCopy) {   // this block wrote _nxt itself (act_body, block 0)
      SWARM_RTSTAMP(17);
      for (int i = threadIdx.x; i < N_PARAMS_PAD; i += 256) {
        R.lr.w_cur[i] = R.lr.w_nxt[i];
        R.lr.m_cur[i] = R.lr.m_nxt[i];
        R.lr.v_cur[i] = R.lr.v_nxt[i];
      }
      SWARM_RTSTAMP(19);
      return;
    }
    if (threadIdx.x == 0)   // every block read this epoch at its start: the next launch counts afresh
      __hip_atomic_store(R.ws + kWsEpoch, epoch + 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    SWARM_RTSTAMP(17);
    red_control(C, R.ctl);
    SWARM_RTSTAMP(19);
    return;
  }
  // ---- column role: columns cb * 16 + c; thread (c, q) owns groups 4q .. 4q + 3
  const int cb = vb - kRedRoleCol0;
  const int c = threadIdx.x % kRedCols, q = threadIdx.x / kRedCols;
  const int col = cb * kRedCols + c;
  const int per = (R.n_slabs + kRedGroups - 1) / kRedGroups;   // <= kRedMaxPer (host check)
  const uint32_t tag = tick + 1u;
  float val[4 * kRedMaxPer];
  uint32_t need = 0u;
#pragma unroll
  for (int i = 0; i < 4 * kRedMaxPer; ++i) {
    val[i] = 0.0f;
    const int b = (4 * q + i / kRedMaxPer) * per + i % kRedMaxPer;
    if (col <= N_PARAMS && i % kRedMaxPer < per && b < R.n_slabs) need |= 1u << i;
  }
  red_wait(R.ws + kWsTdDone, epoch, n_td > SWARM_RED_LEAD ? n_td - SWARM_RED_LEAD : 0u, R.err);
  SWARM_RTSTAMP(17);
  for (int spin = 0;; ++spin) {
    // two halves of 16 granules (64 VGPRs of loads in flight, not 128: the 16-slot tick kernel
    // runs at 3 waves per SIMD)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      constexpr int kH = 2 * kRedMaxPer;
      unsigned long long g[kH];
#pragma unroll
      for (int u = 0; u < kH; ++u) {   // every missing granule's load in flight at once
        const int i = h * kH + u;
        const int b = (4 * q + i / kRedMaxPer) * per + i % kRedMaxPer;
        g[u] = 0ull;
        if ((need >> i) & 1u) g[u] = ld_granule(R.slabs + slab_index(col, b, R.n_slabs));
      }
#pragma unroll
      for (int u = 0; u < kH; ++u) {
        const int i = h * kH + u;
        if (((need >> i) & 1u) && (uint32_t)(g[u] >> 32) == tag) {
          val[i] = __uint_as_float((uint32_t)g[u]);
          need &= ~(1u << i);
        }
      }
    }
    if (!__builtin_amdgcn_ballot_w64(need != 0u)) break;
    if (spin >= kHoSpinLimit) {   // never in a correct run: count it; the missing terms stay 0
      if ((threadIdx.x & 63) == 0) atomicAdd(R.err, 1u);
      break;
    }
    __builtin_amdgcn_s_sleep(SWARM_RED_SLEEP);
  }
  SWARM_RTSTAMP(18);
  // group sums in grad_reduce_kernel's order: s = v[b0], then + v[b0 + j] (0 past the group)
#pragma unroll
  for (int gi = 0; gi < 4; ++gi) {
    const int b0 = (4 * q + gi) * per, b1 = min(R.n_slabs, b0 + per);
    float v0[kRedChunk];
#pragma unroll
    for (int j = 0; j < kRedChunk; ++j) v0[j] = (col <= N_PARAMS && b0 + j < b1) ? val[gi * kRedMaxPer + j] : 0.0f;
    float s = v0[0];
#pragma unroll
    for (int j = 1; j < kRedChunk; ++j) s = s + v0[j];
    L.part[4 * q + gi][c] = s;
  }
  __syncthreads();
  if (q < kRedRuns) {
    float r = L.part[8 * q][c];
#pragma unroll
    for (int gi = 1; gi < 8; ++gi) r = r + L.part[8 * q + gi][c];
    L.part2[q][c] = r;
  }
  __syncthreads();
  if (q == 0 && col <= N_PARAMS) {
    float tot = L.part2[0][c];
#pragma unroll
    for (int gi = 1; gi < kRedRuns; ++gi) tot = tot + L.part2[gi][c];
    R.grad[col] = tot;
    if (col == N_PARAMS) C->loss = tot / (float)((size_t)R.ctl.batch * R.N);
  }
  SWARM_RTSTAMP(19);
}

}  // namespace swarm
