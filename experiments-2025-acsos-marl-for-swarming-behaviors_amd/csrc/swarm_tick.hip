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

namespace swarm {

template <int NSA, int NST>
union TickSmem {
  ActSmem<NSA> a;
  TdSmem<NST> t;
};

// Occupancy target: with N <= 8 (GS = 8) the grid is 2 blocks per CU at C2 (512 blocks, 256
// CUs), so 2 waves per SIMD is all it needs, and at that target the compiler keeps the MFMA
// accumulators in ArchVGPRs (no AGPR copies): 15.22 -> 15.07 us per tick (profiles/r02_ab_wpe.jsonl).
// N > 8 (one graph per TD wave) keeps 3: C3's 768 blocks must all be resident.
template <int NSA, int NST, int GS, int SCEN, int SPEC>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(GS == 8 ? 2 : 3, GS == 8 ? 2 : 3))) void tick_kernel(const swarm_ctrl* __restrict__ ctrl, float* state,
                                                   const float* grad, const float* w_cur, const float* m_cur,
                                                   const float* v_cur, int B, int N, ActArgs A,
                                                   TdArgs T, TdFused X) {
  static_assert(64 * kActWPB == 256 && 128 * (kTdRows / NST) == 256, "one block shape for both halves");
  __shared__ TickSmem<NSA, NST> U;
  // every argument the first round trip needs arrives preloaded in SGPRs (the leading 14
  // dwords); the acting/TD split is derived from B instead of a 15th kernel argument
  const int n_act = (B + kActWPB - 1) / kActWPB;
  if ((int)blockIdx.x < n_act) {
    act_body<NSA, MODE_TICK, SCEN, SPEC, true, SWARM_NET_GCN>(U.a, blockIdx.x, n_act, ctrl, state, grad, w_cur, m_cur,
                                                              v_cur, B, N, A);
  } else {
    td_body<NST, GS, SPEC, true>(U.t, (int)blockIdx.x - n_act, nullptr, T.replay.s, T.replay.s_next, T.replay.r,
                                      T.replay.a, T.S, B, N, T.replay.capacity, T, X, ctrl, grad, w_cur, m_cur, v_cur);
  }
}

}  // namespace swarm

using namespace swarm;

namespace {
// workspace: [err: 1 u32, padded to 512 B], then the tagged hand-off records
size_t err_bytes() { return 512; }
size_t rec_bytes(int B, int N) { return (size_t)B * ho_stride_granules(N) * 8; }
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
  const dim3 grid(n_act + n_td), block(256);
  hipStream_t st = (hipStream_t)stream;
  const float *g = lr->grad, *w = lr->w_cur, *m = lr->m_cur, *v = lr->v_cur;
  const bool oa = cfg->scenario == SWARM_OBSTACLE_AVOIDANCE;
  // complete graph (the reference's training graph) and GoTo's radius graph with GAT (the
  // north_star graph, N <= 8): graph and conv fixed at compile time; others: the
  // runtime-switched kernel
  const int spec = spec_of(cfg->graph, cfg->conv);
#define SWARM_TICK_LAUNCH(NSA, GS, SC, SP)                                                                      \
  hipLaunchKernelGGL((tick_kernel<NSA, 16, GS, SC, SP>), grid, block, 0, st, ctrl, state, g, w, m, v, B, N, a, t, x)
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
