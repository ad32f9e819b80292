// swarm_td.hip — learning side of the hot path: replay sample, TD loss, hand-written
// backward through GCN (PyG GATConv + MLP), deterministic gradient reduction,
// clip_grad_norm_ and Adam.  gfx950 only.
//
// Reference: DQNTrainer.train_step_dqn (src/training/train_gcn_dqn.py:112-137),
// GraphReplayBuffer.sample (:38-45), Adam(lr=1e-3) (:85), target sync (:131-133).
#include <stdlib.h>

#include "swarm_tdk.h"
#include "swarm_peer.h"

namespace swarm {

// One TD block = 32 node slots (swarm_tdk.h).  The dependent chain's pointers (batch indices
// -> replay rows) and the geometry lead the parameter list: preloaded into SGPRs (kernarg
// preload), the index loads issue at wave start.
template <int NS, int GS, int SPEC>
__global__ __launch_bounds__(128 * (kTdRows / NS)) void td_kernel(const int32_t* sample_in, const float* rs,
                                                                  const float* rs_next, const float* rr,
                                                                  const uint8_t* ra, int S, int B, int N,
                                                                  int capacity, TdArgs A) {
  __shared__ TdSmem<NS> L;
  td_body<NS, GS, SPEC>(L, blockIdx.x, sample_in, rs, rs_next, rr, ra, S, B, N, capacity, A, TdFused{});
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
  swarm_peer peer;        // PEER = 1: the all-reduce over the ranks' exchange buffers (swarm_peer.h)
};

// 1024 threads = 16 columns x 64 slab groups (105 column blocks: the 1.7 MB of freshly
// written slabs is read by many CUs at once, 16 KB each); group g sums a contiguous run of
// slabs with every load issued before the ordered adds, then the 64 group sums of a column
// are added in a fixed two-level order (8 runs of 8, then the 8 run sums): bitwise
// reproducible run to run.  Advance mode adds one control block (the last): it prepares
// and stores the whole ctrl update (Adam scalars of the next step in double, the next
// tick's sampling key) in parallel with the column blocks, so no column block waits on it.
// Three more blocks copy w / m / v _nxt -> _cur (one array each), beside the column blocks.
#ifndef SWARM_RED_GROUPS
#define SWARM_RED_GROUPS 64   // test builds: 16 (256-thread blocks, so 8 ranks' peer reduces fit one GPU)
#endif
constexpr int kRedCols = 16;      // columns per reduce block
constexpr int kRedGroups = SWARM_RED_GROUPS;   // slab groups per column (consecutive slabs each)
constexpr int kRedRuns = kRedGroups / 8;
constexpr int kRedChunk = 8;      // slabs per load chunk of a group
constexpr int kRedColBlocks = (N_PARAMS + 1 + kRedCols - 1) / kRedCols;
constexpr int kRedCopyBlocks = 3;

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
      b1p = b1p * adam_beta1(A.hp);
      b2p = b2p * adam_beta2(A.hp);
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
    // (float)(1 - beta) of the Adam step, rewritten every tick from the launch's double
    // hyper-parameters: a control block that skipped swarm_ctrl_init (zero-filled) has its
    // first optimizer step pending only after this write, so no step runs with 0 here
    C->one_m_beta1 = (float)(1.0 - adam_beta1(A.hp));
    C->one_m_beta2 = (float)(1.0 - adam_beta2(A.hp));
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

static_assert(kRedGroups % 8 == 0 && kRedCols * kRedGroups <= 1024, "reduce geometry");
static_assert(kRedColBlocks <= kPeerSeqRegion, "peer seq region");
static_assert(kRedColBlocks == kGradSqCount && kRedCols == 16, "one norm partial per column block");
// slabs / ctrl / geometry preloaded into SGPRs (kernarg preload): the slab loads issue at wave start.
// PEER = 1 (swarm_reduce_advance_peer): each column block then exchanges its 16 column sums with
// the other ranks (swarm_peer.h) and writes grad = their rank-ordered sum: the all-reduce costs
// one xGMI store + poll inside this launch instead of a collective launch after it.
template <int PEER>
__global__ __launch_bounds__(kRedCols * kRedGroups) void grad_reduce_kernel(const float* slabs, swarm_ctrl* ctrl,
                                                                            int n_slabs, int advance, ReduceArgs A) {
  __shared__ float part[kRedGroups][kRedCols];
  __shared__ float part2[kRedRuns][kRedCols];
  __shared__ float peer_rv[PEER ? SWARM_PEER_MAX : 1][kRedCols];
  __shared__ float sqv[kRedCols];
  SWARM_RTSTAMP(22);
  SWARM_STAMP(28);
  swarm_ctrl* C = ctrl;
  if ((int)blockIdx.x > kRedColBlocks) {   // advance mode: a copy-back block
    const int j = (int)blockIdx.x - kRedColBlocks - 1;
    const float4* src = reinterpret_cast<const float4*>(j == 0 ? A.lr.w_nxt : (j == 1 ? A.lr.m_nxt : A.lr.v_nxt));
    float4* dst = reinterpret_cast<float4*>(j == 0 ? A.lr.w_cur : (j == 1 ? A.lr.m_cur : A.lr.v_cur));
    if ((int)threadIdx.x < N_PARAMS_PAD / 4) dst[threadIdx.x] = src[threadIdx.x];
    return;
  }
  if ((int)blockIdx.x == kRedColBlocks) {   // advance mode: the control block (red_control)
    RedCtrl rc;
    rc.capacity = A.capacity; rc.B = A.B; rc.batch = A.batch; rc.hp = A.hp; rc.k0 = A.k0; rc.k1 = A.k1;
    red_control(C, rc);
    return;
  }
  const int c = threadIdx.x % kRedCols;
  const int col = blockIdx.x * kRedCols + c;
  const int q = threadIdx.x / kRedCols;
  const int per = (n_slabs + kRedGroups - 1) / kRedGroups;
  const int b0 = q * per, b1 = min(n_slabs, b0 + per);
  // first chunk of this thread's slab column in flight before anything else.  Column col of
  // slab b is scol[16 b] (swarm_common.h slab_index): one 64-bit base per thread, 32-bit offsets
  constexpr int kChunk = kRedChunk;
  static_assert(kSlabCols == 16, "slab column blocks of 16");
  const float* const scol = slabs + ((size_t)(col >> 4) * (size_t)n_slabs * kSlabCols + (size_t)(col & 15));
  float v0[kChunk];
#pragma unroll
  for (int j = 0; j < kChunk; ++j)
    v0[j] = (col <= N_PARAMS && b0 + j < b1) ? scol[(uint32_t)(b0 + j) * kSlabCols] : 0.0f;
  float s = v0[0];
#pragma unroll
  for (int j = 1; j < kChunk; ++j) s = s + v0[j];
  if (col <= N_PARAMS) {
    for (int b = b0 + kChunk; b < b1; b += kChunk) {
      float v[kChunk];
#pragma unroll
      for (int j = 0; j < kChunk; ++j) v[j] = (b + j < b1) ? scol[(uint32_t)(b + j) * kSlabCols] : 0.0f;
#pragma unroll
      for (int j = 0; j < kChunk; ++j) s = s + v[j];
    }
  }
  SWARM_STAMP(29);
  part[q][c] = s;
  __syncthreads();
  SWARM_STAMP(30);
  if (q < kRedRuns) {
    float r = part[8 * q][c];
#pragma unroll
    for (int gi = 1; gi < 8; ++gi) r = r + part[8 * q + gi][c];
    part2[q][c] = r;
  }
  __syncthreads();
  float gcol = 0.0f;   // q == 0: this column's gradient as written to grad
  if (q == 0 && col <= N_PARAMS) {
    float tot = part2[0][c];
#pragma unroll
    for (int gi = 1; gi < kRedRuns; ++gi) tot = tot + part2[gi][c];
    if (PEER) part[0][c] = tot;   // part[0] is free again: this rank's column sums
    else A.grad[col] = tot;
    gcol = tot;
    // this rank's loss of the update (0 when skipped: the TD launch wrote zero slabs)
    if (advance && col == N_PARAMS) C->loss = tot / (float)((size_t)A.batch * A.N);
  }
  if (PEER) {
    __syncthreads();
    peer_exchange<kRedCols>(A.peer, 0, blockIdx.x, q, c, col, N_PARAMS + 1, part[0], peer_rv, &C->peer_hold);
    if (q == 0 && col <= N_PARAMS) {
      float tot = peer_rv[0][c];
      for (int w = 1; w < A.peer.world_size; ++w) tot = tot + peer_rv[w][c];
      A.grad[col] = tot;
      gcol = tot;
    }
  }
  // the clip norm's partial of these 16 columns = parameter group blockIdx.x (swarm_adam.h):
  // lanes 0-15 of wave 0 hold the columns; squares as the optimizer step forms them (scaled by
  // 1/W first when W > 1), the float4 sums ((a + b) + c) + d by lanes 0-3, then their quad sum
  if (q == 0) {
    float g = col < N_PARAMS ? gcol : 0.0f;
    if (A.hp.world_size > 1) g = g * (1.0f / (float)A.hp.world_size);
    sqv[c] = g * g;
  }
  wave_lds_sync();   // sqv is written and read by wave 0 only
  if (threadIdx.x < 4) {
    const int f = threadIdx.x;
    const float d = ((sqv[4 * f] + sqv[4 * f + 1]) + sqv[4 * f + 2]) + sqv[4 * f + 3];
    const float sq = quad_sum(d);
    if (f == 0) A.grad[kGradSqBase + blockIdx.x] = sq;
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
  __shared__ float red[64];
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
  // ctrl words 24-25 (swarm_ctrl_init); a control block that skipped it holds 0 there: the
  // same value from the launch's hyper-parameters instead of freezing m and v
  const float one_m_b1 = C->one_m_beta1 != 0.0f ? C->one_m_beta1 : (float)(1.0 - adam_beta1(A.hp));
  const float one_m_b2 = C->one_m_beta2 != 0.0f ? C->one_m_beta2 : (float)(1.0 - adam_beta2(A.hp));
  const bool train = A.flush ? (C->trained != 0u && C->peer_hold == 0u)
                             : (valid_slots * (uint32_t)A.B >= (uint32_t)A.hp.batch);
  // target sync: unfused = after the TD step of tick `tick` ((tick+1) % every); flush = the
  // fused tick already advanced ctrl, so the pending update belongs to tick - 1
  const bool sync = ((A.flush ? tick : tick + 1) % (uint32_t)A.hp.update_target_every) == 0u;
  __syncthreads();   // every thread has read ctrl before thread 0 rewrites it
  float gn = 0.0f;
  if (train) {
    gn = adam_apply(R, A.hp, step_size, inv_bc2, one_m_b1, one_m_b2, tid, red);
    store4(A.params, R.w, R.wt, tid);
    store4(A.m, R.m, R.mt, tid);
    store4(A.v, R.v, R.vt, tid);
    if (sync) store4(A.target, R.w, R.wt, tid);
  }
  if (tid == 0) {
    if (train) {
      C->adam_step = step;
      C->grad_norm = gn;
      ctrl_set_double(C, CTRL_B1POW, ctrl_get_double(C, CTRL_B1POW) * adam_beta1(A.hp));
      ctrl_set_double(C, CTRL_B2POW, ctrl_get_double(C, CTRL_B2POW) * adam_beta2(A.hp));
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
  C->one_m_beta1 = (float)(1.0 - adam_beta1(hp));   // torch: 1 - beta of Python floats
  C->one_m_beta2 = (float)(1.0 - adam_beta2(hp));
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
  if (c->graph < 0 || c->graph > 3) return SWARM_E_BADARG;
  if (c->net != SWARM_NET_GCN) return SWARM_E_UNSUPPORTED;   // GAT3: forward only
  if (c->graph == SWARM_GRAPH_KNN && (c->knn_k < 1 || c->knn_k > c->n_agents)) return SWARM_E_KNN_K;
  if (c->graph == SWARM_GRAPH_RADIUS && !(c->radius > 0.0f)) return SWARM_E_BADARG;
  if (hp->world_size < 1 || hp->update_target_every < 1) return SWARM_E_BADARG;
  return 0;
}
}  // namespace

extern "C" {

int64_t swarm_td_workspace_floats(const swarm_config* cfg, int32_t batch) {
  if (!cfg || cfg->n_agents < 1 || cfg->n_agents > 32 || batch < 1) return SWARM_E_BADARG;
  return (int64_t)(td_max_blocks(cfg, batch) * slab_floats_per_block());
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
  a.radius = cfg->radius;
  a.params = params; a.target = target; a.replay = *replay; a.ctrl = ctrl;
  a.sample_in = sample_in; a.sample_out = sample_out; a.slabs = slabs;
  a.gamma = hp->gamma;
  a.grad_scale = (float)(2.0 / ((double)hp->batch * (double)cfg->n_agents));
  const int nb = td_blocks(cfg, hp->batch);
  a.n_slabs = nb;
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
  hipLaunchKernelGGL(grad_reduce_kernel<0>, dim3(kRedColBlocks), dim3(kRedCols * kRedGroups), 0,
                     (hipStream_t)stream, a.slabs, a.ctrl, a.n_slabs, a.advance, a);
  return (int)hipGetLastError();
}

static int reduce_advance(const swarm_config* cfg, const swarm_adam_cfg* hp, const float* slabs, const swarm_learner* lr,
                          int32_t replay_capacity, swarm_ctrl* ctrl, const swarm_peer* peer, void* stream) {
  if (int e = check_td(cfg, hp)) return e;
  if (!lr || !ctrl || replay_capacity < 1) return SWARM_E_BADARG;
  ReduceArgs a = {};
  if (peer) a.peer = *peer;
  a.n_slabs = td_blocks(cfg, hp->batch); a.slabs = slabs; a.grad = lr->grad;
#if SWARM_DIAG_FEWSLABS   // diagnostic builds only: the reduce reads K slabs (timing bound of a slab cut)
  a.n_slabs = a.n_slabs < SWARM_DIAG_FEWSLABS ? a.n_slabs : SWARM_DIAG_FEWSLABS;
#endif
  a.advance = 1; a.lr = *lr; a.ctrl = ctrl;
  a.capacity = replay_capacity; a.B = cfg->n_envs; a.N = cfg->n_agents; a.batch = hp->batch;
  a.hp = *hp;
  a.k0 = (uint32_t)(cfg->seed & 0xFFFFFFFFu) ^ ((uint32_t)cfg->env_offset * 0x9E3779B9u);
  a.k1 = (uint32_t)(cfg->seed >> 32);
  if (peer)
    hipLaunchKernelGGL(grad_reduce_kernel<1>, dim3(kRedColBlocks + 1 + kRedCopyBlocks), dim3(kRedCols * kRedGroups), 0,
                       (hipStream_t)stream, a.slabs, a.ctrl, a.n_slabs, a.advance, a);
  else
    hipLaunchKernelGGL(grad_reduce_kernel<0>, dim3(kRedColBlocks + 1 + kRedCopyBlocks), dim3(kRedCols * kRedGroups), 0,
                       (hipStream_t)stream, a.slabs, a.ctrl, a.n_slabs, a.advance, a);
  return (int)hipGetLastError();
}

int swarm_reduce_advance(const swarm_config* cfg, const swarm_adam_cfg* hp, const float* slabs, const swarm_learner* lr,
                         int32_t replay_capacity, swarm_ctrl* ctrl, void* stream) {
  return reduce_advance(cfg, hp, slabs, lr, replay_capacity, ctrl, nullptr, stream);
}

int swarm_reduce_advance_peer(const swarm_config* cfg, const swarm_adam_cfg* hp, const float* slabs,
                              const swarm_learner* lr, int32_t replay_capacity, swarm_ctrl* ctrl,
                              const swarm_peer* peer, void* stream) {
  if (int e = check_peer(peer)) return e;
  if (hp && hp->world_size != peer->world_size) return SWARM_E_BADARG;
  return reduce_advance(cfg, hp, slabs, lr, replay_capacity, ctrl, peer, stream);
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
