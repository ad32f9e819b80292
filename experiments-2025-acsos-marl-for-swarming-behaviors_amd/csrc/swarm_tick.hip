// swarm_tick.hip — the fused training tick: the acting blocks and the TD blocks of one
// tick in ONE launch, followed by swarm_reduce_advance (2 launches per tick instead of 3).
// gfx950 only.
//
// Reference: the hot loop of DQNTrainer.train_model (src/training/train_gcn_dqn.py:153-178):
//   graph -> model -> eps-greedy -> env.step -> replay.push -> train_step_dqn (:112-137).
//
// Blocks [0, n_act) are acting blocks (swarm_actk.h, one env per wave); blocks
// [n_act, n_act + n_td) are TD blocks (swarm_tdk.h).  Both apply the pending optimizer step
// of the previous tick in registers, so neither waits on a launch boundary for the weights.
// The only in-launch dependency is the reference's push-then-sample order: a TD graph drawn
// from THIS tick's replay slot waits for the acting wave of its env, which publishes the
// transition as tagged write-through granules (swarm_common.h).  Acting blocks never wait
// and have the lower block indices; the wait is bounded (kHoSpinLimit) and counted in the
// workspace's error word, so the grid always drains.  Every other TD graph (slots written by
// earlier ticks) runs concurrently with acting.
#include "swarm_actk.h"
#include "swarm_tdk.h"
#include "swarm_red.h"

// A/B knob (tools/ab_build.py only; 0 in every shipped library): TD blocks sleep
// SWARM_TD_DELAY x 1024 cycles before their first loads, so the acting blocks' prologue
// (the hand-off graphs' critical path) has the memory system to itself
#ifndef SWARM_TD_DELAY
#define SWARM_TD_DELAY 0
#endif

namespace swarm {

template <int NSA, int NST>
union TickSmem {
  ActSmem<NSA> a;
  TdSmem<NST> t;
  RedSmem r;   // one-launch tick: an acting block's reduce role, after its env is stepped
};

// Occupancy target: with N <= 8 (GS = 8) the grid is 2 blocks per CU at C2 (512 blocks, 256
// CUs), so 2 waves per SIMD is all it needs, and at that target the compiler keeps the MFMA
// accumulators in ArchVGPRs (no AGPR copies): 15.22 -> 15.07 us per tick (profiles/r02_ab_wpe.jsonl).
// N > 8 (one graph per TD wave) keeps 3: C3's 768 blocks must all be resident.
template <int NSA, int NST, int GS, int SCEN, int SPEC, bool RED = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(GS == 8 ? 2 : 3, GS == 8 ? 2 : 3))) void tick_kernel(const swarm_ctrl* __restrict__ ctrl, float* state,
                                                   const float* grad, const float* w_cur, const float* m_cur,
                                                   const float* v_cur, int B, int N, ActArgs A,
                                                   TdArgs T, TdFused X, RedTick Rt) {
  static_assert(64 * kActWPB == 256 && 128 * (kTdRows / NST) == 256, "one block shape for both halves");
  __shared__ TickSmem<NSA, NST> U;
  // every argument the first round trip needs arrives preloaded in SGPRs (the leading 14
  // dwords); the acting/TD split is derived from B instead of a 15th kernel argument
  const int n_act = (B + kActWPB - 1) / kActWPB;
  if ((int)blockIdx.x < n_act) {
    // RED: this launch's tick and epoch, read with the prologue's ctrl line (the control role
    // rewrites both later)
    const uint32_t tick0 = RED ? ctrl->tick : 0u;
    const unsigned long long epoch0 = RED ? red_epoch_load(Rt.ws) : 0ull;
    act_body<NSA, MODE_TICK, SCEN, SPEC, true, SWARM_NET_GCN, RED>(U.a, blockIdx.x, n_act, ctrl, state, grad, w_cur,
                                                                  m_cur, v_cur, B, N, A);
    if constexpr (RED) {
      if ((int)blockIdx.x < kRedRoles) red_role((int)blockIdx.x, Rt, const_cast<swarm_ctrl*>(ctrl), tick0, epoch0, U.r);
    }
  } else {
    for (int i = 0; i < SWARM_TD_DELAY; ++i) __builtin_amdgcn_s_sleep(16);
    td_body<NST, GS, SPEC, true, RED>(U.t, (int)blockIdx.x - n_act, nullptr, T.replay.s, T.replay.s_next, T.replay.r,
                                      T.replay.a, T.S, B, N, T.replay.capacity, T, X, ctrl, grad, w_cur, m_cur, v_cur);
  }
}

}  // namespace swarm

using namespace swarm;

namespace {
// workspace: [err: 1 u32 | the one-launch tick's epoch | its two counters (swarm_common.h kWs*):
// one 128-B line each], then the tagged hand-off records
size_t err_bytes() { return 512; }
size_t rec_bytes(int B, int N) { return (size_t)B * ho_stride_granules(N) * 8; }

// RED (one launch per tick) exists for the 8-slot kernels (n_agents <= 8): the 16-slot kernel's
// 3 waves per SIMD leave too few VGPRs for the column roles' granule sweep
template <int NSA, int GS, int SC, int SP>
void tick_launch(bool red, dim3 grid, dim3 block, hipStream_t st, const swarm_ctrl* ctrl, float* state, const float* g,
                 const float* w, const float* m, const float* v, int B, int N, const ActArgs& a, const TdArgs& t,
                 const TdFused& x, const RedTick& rt) {
  if constexpr (NSA == 8) {
    if (red) {
      hipLaunchKernelGGL((tick_kernel<NSA, 16, GS, SC, SP, true>), grid, block, 0, st, ctrl, state, g, w, m, v, B, N, a, t,
                         x, rt);
      return;
    }
  }
  hipLaunchKernelGGL((tick_kernel<NSA, 16, GS, SC, SP>), grid, block, 0, st, ctrl, state, g, w, m, v, B, N, a, t, x, rt);
}
}  // namespace

extern "C" {

int swarm_train_tick_supported(const swarm_config* cfg) {
  if (!cfg || cfg->n_agents < 1 || cfg->n_agents > 16 || cfg->n_envs < 1 || cfg->net != SWARM_NET_GCN) return 0;
  if (cfg->graph == SWARM_GRAPH_KNN && (cfg->knn_k < 1 || cfg->knn_k > cfg->n_agents)) return 0;
  if (cfg->graph == SWARM_GRAPH_RADIUS && !(cfg->radius > 0.0f)) return 0;
  return (cfg->graph == SWARM_GRAPH_COMPLETE || cfg->graph == SWARM_GRAPH_KNN || cfg->graph == SWARM_GRAPH_RADIUS) &&
         (cfg->conv == SWARM_CONV_GAT || cfg->conv == SWARM_CONV_GCN) &&
         (cfg->scenario == SWARM_GOTO || cfg->scenario == SWARM_OBSTACLE_AVOIDANCE ||
          (cfg->scenario == SWARM_FLOCKING && cfg->n_agents >= 2));
}

int swarm_train_tick_reduce_supported(const swarm_config* cfg, const swarm_adam_cfg* hp) {
  if (!cfg || !hp || !swarm_train_tick_supported(cfg) || hp->world_size != 1 || cfg->n_agents > 8) return 0;
  const int n_act = (cfg->n_envs + kActWPB - 1) / kActWPB;
  const int gs = cfg->n_agents <= 8 ? 8 : 16;
  const int n_td = (hp->batch + (kTdRows / gs) - 1) / (kTdRows / gs);
  return n_act >= kRedRoles && n_td <= kRedGroups * kRedMaxPer;
}

int64_t swarm_train_tick_workspace_bytes(const swarm_config* cfg) {
  if (!swarm_train_tick_supported(cfg)) return SWARM_E_UNSUPPORTED;
  return (int64_t)(err_bytes() + rec_bytes(cfg->n_envs, cfg->n_agents));
}

int swarm_train_tick(const swarm_config* cfg, const swarm_adam_cfg* hp, const swarm_learner* lr, float* state,
                     const swarm_replay* replay, const swarm_ctrl* ctrl, const swarm_act_out* out, float* slabs,
                     void* workspace, int32_t* sample_out, void* stream) {
  if (!cfg || !hp || !lr || !replay || !ctrl || !slabs || !workspace || !state) return SWARM_E_BADARG;
  if (!swarm_train_tick_supported(cfg)) return SWARM_E_UNSUPPORTED;
  if (hp->batch < 1 || hp->world_size < 1 || hp->update_target_every < 1 || replay->capacity < 1 || !replay->s)
    return SWARM_E_BADARG;
  const int B = cfg->n_envs, N = cfg->n_agents;
  char* ws = static_cast<char*>(workspace);
  uint32_t* err = reinterpret_cast<uint32_t*>(ws);
  unsigned long long* rec = reinterpret_cast<unsigned long long*>(ws + err_bytes());

  ActArgs a = {};
  a.B = B; a.N = N; a.scenario = cfg->scenario; a.graph = cfg->graph; a.k = cfg->knn_k; a.conv = cfg->conv;
  a.env_offset = cfg->env_offset; a.flags = cfg->flags;
  a.k0 = (uint32_t)(cfg->seed & 0xFFFFFFFFu); a.k1 = (uint32_t)(cfg->seed >> 32); a.radius = cfg->radius;
  a.state = state; a.ctrl = ctrl; a.learn = 1; a.lr = *lr; a.hp = *hp; a.sample_out = nullptr;
  a.grad_norm_out = const_cast<float*>(&ctrl->grad_norm);
  a.replay = *replay;
  if (out) a.out = *out;
  a.ho_rec = rec;

  TdArgs t = {};
  t.S = hp->batch; t.B = B; t.N = N; t.graph = cfg->graph; t.k = cfg->knn_k; t.conv = cfg->conv;
  t.env_offset = cfg->env_offset; t.k0 = a.k0; t.k1 = a.k1; t.radius = cfg->radius;
  t.params = lr->w_nxt; t.target = lr->target; t.replay = *replay; t.ctrl = ctrl;
  t.sample_in = nullptr; t.sample_out = sample_out; t.slabs = slabs;
  t.gamma = hp->gamma;
  t.grad_scale = (float)(2.0 / ((double)hp->batch * (double)N));

  TdFused x = {};
  x.lr = *lr; x.hp = *hp; x.ho_rec = rec; x.ho_err = err;

  const int n_act = (B + kActWPB - 1) / kActWPB;
  const int gs = N <= 8 ? 8 : 16;
  const int n_td = (hp->batch + (kTdRows / gs) - 1) / (kTdRows / gs);
  t.n_slabs = n_td;
  // one launch per tick (swarm_red.h): the reduce and the ctrl advance run in this launch
  const bool red = (cfg->flags & SWARM_F_TICK_REDUCE) != 0;
  RedTick rt = {};
  if (red) {
    if (!swarm_train_tick_reduce_supported(cfg, hp)) return SWARM_E_UNSUPPORTED;
    unsigned long long* ws64 = reinterpret_cast<unsigned long long*>(ws);
    a.red_ws = ws64; x.red_ws = ws64;
    rt.ws = ws64; rt.err = err; rt.slabs = reinterpret_cast<const unsigned long long*>(slabs);
    rt.n_slabs = n_td; rt.n_act = n_act; rt.grad = lr->grad; rt.lr = *lr; rt.N = N;
    rt.ctl.capacity = replay->capacity; rt.ctl.B = B; rt.ctl.batch = hp->batch; rt.ctl.hp = *hp;
    rt.ctl.k0 = (uint32_t)(cfg->seed & 0xFFFFFFFFu) ^ ((uint32_t)cfg->env_offset * 0x9E3779B9u);
    rt.ctl.k1 = (uint32_t)(cfg->seed >> 32);
  }
  const dim3 grid(n_act + n_td), block(256);
  hipStream_t st = (hipStream_t)stream;
  const float *g = lr->grad, *w = lr->w_cur, *m = lr->m_cur, *v = lr->v_cur;
  const bool oa = cfg->scenario == SWARM_OBSTACLE_AVOIDANCE;
  // complete graph (the reference's training graph) and GoTo's radius graph with GAT (the
  // north_star graph, N <= 8): graph and conv fixed at compile time; others: the
  // runtime-switched kernel
  const int spec = spec_of(cfg->graph, cfg->conv);
#define SWARM_TICK_LAUNCH(NSA, GS, SC, SP) \
  tick_launch<NSA, GS, SC, SP>(red, grid, block, st, ctrl, state, g, w, m, v, B, N, a, t, x, rt)
#define SWARM_TICK_LAUNCH2(NSA, GS, SC)                                               \
  do {                                                                                 \
    if (spec == SPEC_COMPLETE_GAT) SWARM_TICK_LAUNCH(NSA, GS, SC, SPEC_COMPLETE_GAT);  \
    else if (spec == SPEC_COMPLETE_GCN) SWARM_TICK_LAUNCH(NSA, GS, SC, SPEC_COMPLETE_GCN); \
    else SWARM_TICK_LAUNCH(NSA, GS, SC, SPEC_RUNTIME);                                 \
  } while (0)
  const bool fl = cfg->scenario == SWARM_FLOCKING;
  if (N <= 8) {
    if (fl) SWARM_TICK_LAUNCH2(8, 8, SWARM_FLOCKING);
    else if (oa) SWARM_TICK_LAUNCH2(8, 8, SWARM_OBSTACLE_AVOIDANCE);
    else if (spec == SPEC_RADIUS_GAT) SWARM_TICK_LAUNCH(8, 8, SWARM_GOTO, SPEC_RADIUS_GAT);
    else SWARM_TICK_LAUNCH2(8, 8, SWARM_GOTO);
  } else {
    if (fl) SWARM_TICK_LAUNCH2(16, 16, SWARM_FLOCKING);
    else if (oa) SWARM_TICK_LAUNCH2(16, 16, SWARM_OBSTACLE_AVOIDANCE);
    else SWARM_TICK_LAUNCH2(16, 16, SWARM_GOTO);
  }
#undef SWARM_TICK_LAUNCH2
#undef SWARM_TICK_LAUNCH
  return (int)hipGetLastError();
}

#if SWARM_STAMPS
int swarm_dbg_stamps_tick(void* p) { return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_swarm_stamps), &p, sizeof(p)); }
#endif

uint32_t swarm_host_sample_index(uint32_t i, uint32_t n, uint32_t k0, uint32_t k1, uint32_t tick) {
  return sample_index(i, sample_key(n, k0, k1, tick));
}
uint32_t swarm_host_sample_position(uint32_t g, uint32_t n, uint32_t k0, uint32_t k1, uint32_t tick) {
  return sample_position(g, sample_key(n, k0, k1, tick));
}

}  // extern "C"
