// swarm_act.hip — acting side of the hot path: reset, env.step, graph build,
// GCN.forward, the fused acting tick and the multi-tick rollout.  gfx950 only.
//
// Reference call sites replaced (paths relative to the reference checkout):
//   train_gcn_dqn.py:161-172   graph -> model -> eps-greedy -> env.step -> replay.push
//   simulator.py:59-93         kNN graph -> argmax -> env.step -> metrics
//   go_to_position_scenario.py:83-132, obstacle_avoidance_scenario.py:94-173
#include <stdlib.h>

#include "swarm_actk.h"

namespace swarm {

// One acting block = kActWPB environments (swarm_actk.h); the first round trip's pointers and
// the geometry lead the parameter list (kernarg preload into SGPRs).
template <int NS, int MODE, int SCEN, int SPEC, int NET = SWARM_NET_GCN>
__global__ __launch_bounds__(64 * kActWPB) void act_kernel(const swarm_ctrl* __restrict__ ctrl, float* state,
                                                          const float* grad, const float* w_cur,
                                                          const float* m_cur, const float* v_cur, int B, int N,
                                                          ActArgs A) {
  __shared__ ActSmem<NS> S;
  act_body<NS, MODE, SCEN, SPEC, false, NET>(S, blockIdx.x, gridDim.x, ctrl, state, grad, w_cur, m_cur, v_cur, B, N, A);
}

// A/B knob: SWARM_ROLLOUT_WPE = w > 0 launches the multi-tick rollouts through this copy of the
// kernel with an occupancy target of w waves per SIMD (the register budget the compiler may
// use); 0 = act_kernel with the compiler's default
#ifndef SWARM_ROLLOUT_WPE
#define SWARM_ROLLOUT_WPE 0
#endif
#if SWARM_ROLLOUT_WPE > 0
template <int NS, int MODE, int SCEN, int SPEC, int NET = SWARM_NET_GCN>
__global__ __launch_bounds__(64 * kActWPB) __attribute__((amdgpu_waves_per_eu(SWARM_ROLLOUT_WPE, SWARM_ROLLOUT_WPE)))
void act_kernel_w(const swarm_ctrl* __restrict__ ctrl, float* state, const float* grad, const float* w_cur,
                  const float* m_cur, const float* v_cur, int B, int N, ActArgs A) {
  __shared__ ActSmem<NS> S;
  act_body<NS, MODE, SCEN, SPEC, false, NET>(S, blockIdx.x, gridDim.x, ctrl, state, grad, w_cur, m_cur, v_cur, B, N, A);
}
#endif

// ---------------------------------------------------------------- reset
// reset_world_at + generate_grid; centre from Philox + Box-Muller (fp32 libm)
__global__ void reset_kernel(int B, int N, int scenario, int flags, uint32_t k0, uint32_t k1, int env_offset,
                             uint32_t episode, float* __restrict__ state) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  const int env = gid / N, agent = gid - env * N;
  if (env >= B) return;
  const uint32_t key_env = (flags & SWARM_F_SHARED_RESET) ? 0u : (uint32_t)(env_offset + env);
  const u32x4 w = philox4x32(episode, key_env, STREAM_RESET, 0u, k0, k1);
  const float u1 = ((float)(w.x >> 8) + 1.0f) * 5.9604644775390625e-08f;
  const float u2 = (float)(w.y >> 8) * 5.9604644775390625e-08f;
  const float rr = sqrtf(-2.0f * logf(u1));
  const float z0 = rr * cosf(6.283185307179586f * u2), z1 = rr * sinf(6.283185307179586f * u2);
  float cx, cy;
  if (scenario == SWARM_GOTO) {
    cx = 1.5f + (-0.6f + 0.4f * z0);
    cy = -1.5f + (0.6f + 0.4f * z1);
  } else if (scenario == SWARM_FLOCKING) {   // flocking_scenario.py:86-91: [-1, 1] + N((-0.6,0.6), 0.4)
    cx = -1.0f + (-0.6f + 0.4f * z0);
    cy = 1.0f + (0.6f + 0.4f * z1);
  } else {
    const float s = (flags & SWARM_F_RANDOM_OA) ? 0.1f : 0.0f;
    cx = 0.6f + s * z0;
    cy = -0.6f + s * z1;
  }
  int cols = 1;
  while (cols * cols < N) ++cols;
  const int rows = (N + cols - 1) / cols;
  const int i = agent / cols, j = agent - i * cols;
  const float ox = (float)(((double)j - (double)(cols - 1) / 2.0) * 0.15);
  const float oy = (float)(((double)i - (double)(rows - 1) / 2.0) * 0.15);
  reinterpret_cast<float4*>(state)[gid] = make_float4(cx + ox, cy + oy, 0.0f, 0.0f);
}

// ---------------------------------------------------------------- scenario state (Flocking)
// previous_distance_to_agents of every agent, from the positions in `state`, into the [B][N]
// floats after it.  fresh != 0: as reset_world_at leaves it (flocking_scenario.py:93-122): the
// loop sets agent i's position and measures it in the same iteration, so agents j > i are still
// where VMAS's World.reset put them (zeroed, before reset_world_at runs); fresh == 0: as a
// reward call leaves it (:151-164), every agent at its current position.  Same operation order
// as act_body's post-step spread.
__global__ void flock_state_kernel(int B, int N, int fresh, float* __restrict__ state) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  const int env = gid / N, i = gid - env * N;
  if (env >= B) return;
  const float4* st = reinterpret_cast<const float4*>(state) + (size_t)env * N;
  const float4 me = st[i];
  float s = 0.0f;
  for (int j = 0; j < N; ++j) {
    if (j == i) continue;
    float qx = 0.0f, qy = 0.0f;
    if (!fresh || j < i) { const float4 o = st[j]; qx = o.x; qy = o.y; }
    const float b = norm2(me.x - qx, me.y - qy) - kFlockDesired;
    s = s + b * b;
  }
  state[(size_t)B * N * 4 + gid] = (s / (float)(N - 1)) * kFlockShaping;
}

// ---------------------------------------------------------------- graph build
template <int NS>
__global__ __launch_bounds__(64) void graph_kernel(ActArgs A, uint8_t* __restrict__ mult_out) {
  __shared__ WSmall<NS> sm;
  __shared__ KV kq[NS][NS];   // per-slot work space of the kNN tie path
  const int N = A.N;
  const WGeom<NS> g = make_wgeom<NS>(blockIdx.x, A.B, N);
  const size_t node = (size_t)g.gid * N + (g.valid ? g.s : 0);
  if (g.q == 0) {
    sm.px[g.s] = g.valid ? A.x[node * kFeat + 0] : 0.0f;
    sm.py[g.s] = g.valid ? A.x[node * kFeat + 1] : 0.0f;
  }
  wave_lds_sync();
  if (A.graph == SWARM_GRAPH_KNN) {
    const uint32_t m = g.valid ? knn_mask<NS>(g, N, A.k, sm, kq[g.s]) : 0u;
    if (g.q == 0) sm.knn[g.s] = m;
    wave_lds_sync();
  } else if (A.graph == SWARM_GRAPH_RADIUS) {
    const uint32_t m = g.valid ? radius_mask_node<NS>(g.s, N, A.radius, sm) : 0u;
    if (g.q == 0) sm.knn[g.s] = m;
    wave_lds_sync();
  }
  int mult[NS];
  in_edges<NS>(g, N, A.graph, sm, nullptr, mult);
  if (g.valid)
    for (int u = g.q; u < N; u += Wpg<NS>::G) mult_out[((size_t)g.gid * N + u) * N + g.s] = (uint8_t)mult[u];
}

// ---------------------------------------------------------------- PyG edge list -> dense multiplicity
// Batch.from_data_list of G graphs of N nodes each (train_gcn_dqn.py:45): node id = g*N + local.
// Counts are packed 4 per 32-bit word and added with integer atomics (order independent).
__global__ void edges_to_mult_kernel(const int64_t* __restrict__ ei, int64_t E, int G, int N,
                                     uint32_t* __restrict__ words, int32_t* __restrict__ err) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= E) return;
  const int64_t s = ei[i], d = ei[E + i];
  const int64_t nn = (int64_t)G * N;
  if (s < 0 || d < 0 || s >= nn || d >= nn || s / N != d / N) { atomicOr(err, 1); return; }
  const int64_t b = s / N;
  const int64_t u = s - b * N, v = d - b * N;
  const int64_t byte = (b * N + u) * N + v;
  atomicAdd(&words[byte >> 2], 1u << (8 * (int)(byte & 3)));
}

}  // namespace swarm

using namespace swarm;

namespace {

int check_cfg(const swarm_config* c) {
  if (!c || c->n_envs < 0 || c->n_agents < 1 || c->n_agents > 32) return SWARM_E_BADARG;
  if (c->scenario != SWARM_GOTO && c->scenario != SWARM_OBSTACLE_AVOIDANCE && c->scenario != SWARM_FLOCKING)
    return SWARM_E_BADARG;
  if (c->scenario == SWARM_FLOCKING && c->n_agents < 2) return SWARM_E_BADARG;   // mean over the other agents
  if (c->net != SWARM_NET_GCN && (c->net != SWARM_NET_GAT3 || c->conv != SWARM_CONV_GAT)) return SWARM_E_BADARG;
  if (c->graph < 0 || c->graph > 3 || (c->conv != SWARM_CONV_GAT && c->conv != SWARM_CONV_GCN)) return SWARM_E_BADARG;
  if (c->graph == SWARM_GRAPH_KNN && (c->knn_k < 1 || c->knn_k > c->n_agents)) return SWARM_E_KNN_K;
  if (c->graph == SWARM_GRAPH_RADIUS && !(c->radius > 0.0f)) return SWARM_E_BADARG;
  return 0;
}

ActArgs make_args(const swarm_config* c) {
  ActArgs a = {};
  a.B = c->n_envs; a.N = c->n_agents; a.scenario = c->scenario; a.graph = c->graph;
  a.k = c->knn_k; a.conv = c->conv; a.env_offset = c->env_offset; a.flags = c->flags;
  a.k0 = (uint32_t)(c->seed & 0xFFFFFFFFu); a.k1 = (uint32_t)(c->seed >> 32);
  a.radius = c->radius;
  a.net = c->net;
  return a;
}

int n_tiles(const swarm_config* c) { return c->n_envs; }   // one wave per environment

template <int MODE>
int launch_act(const ActArgs& a, int tiles, hipStream_t st) {
  if (tiles == 0) return 0;
  const dim3 grid((tiles + kActWPB - 1) / kActWPB), block(64 * kActWPB);
  const float *g = a.lr.grad, *w = a.lr.w_cur, *m = a.lr.m_cur, *v = a.lr.v_cur;
  // specialised kernels for the training tick (complete graph, GAT or GCN) and the rollout
  // (those two plus kNN + GAT, the Simulator's graph, and GoTo's radius + GAT, the north_star
  // graph); everything else runs SPEC_RUNTIME
  constexpr bool kTick = MODE == MODE_TICK || MODE == MODE_ROLLOUT;
  constexpr int S1 = kTick ? SPEC_COMPLETE_GAT : SPEC_RUNTIME;
  constexpr int S2 = kTick ? SPEC_COMPLETE_GCN : SPEC_RUNTIME;
  constexpr int S3 = MODE == MODE_ROLLOUT ? SPEC_KNN_GAT : SPEC_RUNTIME;
  constexpr int S4 = MODE == MODE_ROLLOUT ? SPEC_RADIUS_GAT : SPEC_RUNTIME;   // GoTo, N <= 8 only
  const int spec = kTick ? spec_of(a.graph, a.conv) : SPEC_RUNTIME;
#if SWARM_ROLLOUT_WPE > 0
#define SWARM_ACT_LAUNCH1(NS, SC, SP)                                                                               \
  do {                                                                                                              \
    if constexpr (MODE == MODE_ROLLOUT)                                                                             \
      hipLaunchKernelGGL((act_kernel_w<NS, MODE, SC, SP>), grid, block, 0, st, a.ctrl, a.state, g, w, m, v, a.B, a.N, a); \
    else                                                                                                            \
      hipLaunchKernelGGL((act_kernel<NS, MODE, SC, SP>), grid, block, 0, st, a.ctrl, a.state, g, w, m, v, a.B, a.N, a); \
  } while (0)
#else
#define SWARM_ACT_LAUNCH1(NS, SC, SP) \
  hipLaunchKernelGGL((act_kernel<NS, MODE, SC, SP>), grid, block, 0, st, a.ctrl, a.state, g, w, m, v, a.B, a.N, a)
#endif
#define SWARM_ACT_LAUNCH(NS, SC)                                  \
  do {                                                            \
    if (spec == SPEC_COMPLETE_GAT) SWARM_ACT_LAUNCH1(NS, SC, S1);  \
    else if (spec == SPEC_COMPLETE_GCN) SWARM_ACT_LAUNCH1(NS, SC, S2); \
    else if (spec == SPEC_KNN_GAT) SWARM_ACT_LAUNCH1(NS, SC, S3);  \
    else SWARM_ACT_LAUNCH1(NS, SC, SPEC_RUNTIME);                  \
  } while (0)
  constexpr int OA = (MODE == MODE_Q) ? SWARM_GOTO : SWARM_OBSTACLE_AVOIDANCE;   // MODE_Q has no physics
  constexpr int FL = (MODE == MODE_Q) ? SWARM_GOTO : SWARM_FLOCKING;
  const bool oa = MODE != MODE_Q && a.scenario == SWARM_OBSTACLE_AVOIDANCE;
  const bool fl = MODE != MODE_Q && a.scenario == SWARM_FLOCKING;   // flocking: runtime graph/conv only
  if constexpr (MODE != MODE_STEP) {
  if (a.net == SWARM_NET_GAT3) {   // three-layer GAT (forward only): runtime graph
#define SWARM_ACT_LAUNCH3(NS)                                                                                   \
  do {                                                                                                          \
    if (fl) hipLaunchKernelGGL((act_kernel<NS, MODE, FL, SPEC_RUNTIME, SWARM_NET_GAT3>), grid, block, 0, st,   \
                               a.ctrl, a.state, g, w, m, v, a.B, a.N, a);                                      \
    else if (oa) hipLaunchKernelGGL((act_kernel<NS, MODE, OA, SPEC_RUNTIME, SWARM_NET_GAT3>), grid, block, 0, \
                                    st, a.ctrl, a.state, g, w, m, v, a.B, a.N, a);                             \
    else hipLaunchKernelGGL((act_kernel<NS, MODE, SWARM_GOTO, SPEC_RUNTIME, SWARM_NET_GAT3>), grid, block, 0, \
                            st, a.ctrl, a.state, g, w, m, v, a.B, a.N, a);                                     \
  } while (0)
    if (a.N <= 8) SWARM_ACT_LAUNCH3(8);
    else if (a.N <= 16) SWARM_ACT_LAUNCH3(16);
    else SWARM_ACT_LAUNCH3(32);
#undef SWARM_ACT_LAUNCH3
    return (int)hipGetLastError();
  }
  }
  if (a.N <= 8) {
    if (fl) SWARM_ACT_LAUNCH1(8, FL, SPEC_RUNTIME);
    else if (oa) SWARM_ACT_LAUNCH(8, OA);
    else if (spec == SPEC_RADIUS_GAT) SWARM_ACT_LAUNCH1(8, SWARM_GOTO, S4);
    else SWARM_ACT_LAUNCH(8, SWARM_GOTO);
  } else if (a.N <= 16) {
    if (fl) SWARM_ACT_LAUNCH1(16, FL, SPEC_RUNTIME); else if (oa) SWARM_ACT_LAUNCH(16, OA); else SWARM_ACT_LAUNCH(16, SWARM_GOTO);
  } else {
    if (fl) SWARM_ACT_LAUNCH1(32, FL, SPEC_RUNTIME); else if (oa) SWARM_ACT_LAUNCH(32, OA); else SWARM_ACT_LAUNCH(32, SWARM_GOTO);
  }
#undef SWARM_ACT_LAUNCH
#undef SWARM_ACT_LAUNCH1
  return (int)hipGetLastError();
}

}  // namespace

extern "C" {

int swarm_abi_version(void) { return SWARM_ABI_VERSION; }
int swarm_n_params(void) { return N_PARAMS; }
#ifndef SWARM_SRC_DIGEST
#define SWARM_SRC_DIGEST "unknown"
#endif
#define SWARM_STR2(x) #x
#define SWARM_STR(x) SWARM_STR2(x)
// the build's identity: ABI, the source digest build.py computes over every source, header and
// flag, and the variant knobs; profiles record it (tools/pmc_summary.py) and bench.py uses a
// profile's counters only for the library that wrote them
const char* swarm_build_info(void) {
  return "libswarm_hip gfx950 abi " SWARM_STR(SWARM_ABI_VERSION) " src " SWARM_SRC_DIGEST
#if SWARM_STAMPS == 1
         " stamps"
#elif SWARM_STAMPS == 2
         " rtstamps"
#endif
#if SWARM_HO_FORCE_DROP == 1
         " hodrop"
#elif SWARM_HO_FORCE_DROP == 2
         " hodrop2"
#endif
#ifdef SWARM_RED_GROUPS
         " redgroups" SWARM_STR(SWARM_RED_GROUPS)
#endif
      ;
}

int swarm_env_reset(const swarm_config* cfg, float* state, uint32_t episode, void* stream) {
  if (int e = check_cfg(cfg)) return e;
  const int n = cfg->n_envs * cfg->n_agents;
  if (n == 0) return 0;
  hipLaunchKernelGGL(reset_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, cfg->n_envs,
                     cfg->n_agents, cfg->scenario, cfg->flags, (uint32_t)(cfg->seed & 0xFFFFFFFFu),
                     (uint32_t)(cfg->seed >> 32), cfg->env_offset, episode, state);
  if (cfg->scenario == SWARM_FLOCKING)
    hipLaunchKernelGGL(flock_state_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, cfg->n_envs,
                       cfg->n_agents, 1, state);
  return (int)hipGetLastError();
}

int64_t swarm_state_floats(const swarm_config* cfg) {
  if (int e = check_cfg(cfg)) return e;
  const int64_t n = (int64_t)cfg->n_envs * cfg->n_agents;
  return n * (cfg->scenario == SWARM_FLOCKING ? 5 : 4);
}

int swarm_env_sync_state(const swarm_config* cfg, float* state, int32_t fresh, void* stream) {
  if (int e = check_cfg(cfg)) return e;
  const int n = cfg->n_envs * cfg->n_agents;
  if (n == 0 || cfg->scenario != SWARM_FLOCKING) return 0;
  hipLaunchKernelGGL(flock_state_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, cfg->n_envs,
                     cfg->n_agents, fresh ? 1 : 0, state);
  return (int)hipGetLastError();
}

int swarm_env_step(const swarm_config* cfg, float* state, const int32_t* actions, const swarm_act_out* out,
                   void* stream) {
  if (int e = check_cfg(cfg)) return e;
  if (!actions) return SWARM_E_BADARG;
  ActArgs a = make_args(cfg);
  a.state = state; a.actions = actions;
  if (out) { a.out = *out; a.out.q = nullptr; a.out.mult = nullptr; }
  return launch_act<MODE_STEP>(a, n_tiles(cfg), (hipStream_t)stream);
}

int swarm_build_graph(const swarm_config* cfg, const float* x, uint8_t* mult, void* stream) {
  if (int e = check_cfg(cfg)) return e;
  if (cfg->graph == SWARM_GRAPH_DENSE) return SWARM_E_BADARG;
  ActArgs a = make_args(cfg);
  a.x = x;
  const int tiles = n_tiles(cfg);
  if (tiles == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (a.N <= 8) hipLaunchKernelGGL((graph_kernel<8>), dim3(tiles), dim3(64), 0, st, a, mult);
  else if (a.N <= 16) hipLaunchKernelGGL((graph_kernel<16>), dim3(tiles), dim3(64), 0, st, a, mult);
  else hipLaunchKernelGGL((graph_kernel<32>), dim3(tiles), dim3(64), 0, st, a, mult);
  return (int)hipGetLastError();
}

int swarm_edges_to_mult(const int64_t* edge_index, int64_t n_edges, int32_t n_graphs, int32_t n_nodes,
                        uint8_t* mult, int32_t* err, void* stream) {
  if (!edge_index || !mult || !err || n_graphs < 0 || n_nodes < 1 || n_nodes > 32 || n_edges < 0) return SWARM_E_BADARG;
  if ((reinterpret_cast<uintptr_t>(mult) & 3u) != 0) return SWARM_E_BADARG;
  hipStream_t st = (hipStream_t)stream;
  const size_t bytes = ((size_t)n_graphs * n_nodes * n_nodes + 3) & ~(size_t)3;
  if (hipError_t e = hipMemsetAsync(mult, 0, bytes, st)) return (int)e;
  if (hipError_t e = hipMemsetAsync(err, 0, sizeof(int32_t), st)) return (int)e;
  if (n_edges == 0) return 0;
  hipLaunchKernelGGL(edges_to_mult_kernel, dim3((unsigned)((n_edges + 255) / 256)), dim3(256), 0, st, edge_index,
                     n_edges, n_graphs, n_nodes, reinterpret_cast<uint32_t*>(mult), err);
  return (int)hipGetLastError();
}

int swarm_q_forward(const swarm_config* cfg, const float* params, const float* x, const uint8_t* mult, float* q,
                    void* stream) {
  if (int e = check_cfg(cfg)) return e;
  if (cfg->graph == SWARM_GRAPH_DENSE && !mult) return SWARM_E_BADARG;
  ActArgs a = make_args(cfg);
  a.params = params; a.x = x; a.dense = mult; a.out.q = q;
  return launch_act<MODE_Q>(a, n_tiles(cfg), (hipStream_t)stream);
}

int swarm_act_step(const swarm_config* cfg, const float* params, float* state, const swarm_replay* replay,
                   const swarm_ctrl* ctrl, const swarm_act_out* out, void* stream) {
  if (int e = check_cfg(cfg)) return e;
  if (!ctrl || cfg->graph == SWARM_GRAPH_DENSE) return SWARM_E_BADARG;
  ActArgs a = make_args(cfg);
  a.params = params; a.state = state; a.ctrl = ctrl;
  if (replay) a.replay = *replay;
  if (out) a.out = *out;
  return launch_act<MODE_TICK>(a, n_tiles(cfg), (hipStream_t)stream);
}

int swarm_train_act_step(const swarm_config* cfg, const swarm_adam_cfg* hp, const swarm_learner* lr, float* state,
                         const swarm_replay* replay, const swarm_ctrl* ctrl, const swarm_act_out* out,
                         int32_t* sample_out, void* stream) {
  if (int e = check_cfg(cfg)) return e;
  if (!ctrl || !hp || !lr || cfg->graph == SWARM_GRAPH_DENSE || hp->world_size < 1 || hp->update_target_every < 1)
    return SWARM_E_BADARG;
  if (cfg->net != SWARM_NET_GCN) return SWARM_E_UNSUPPORTED;   // GAT3: forward only
  ActArgs a = make_args(cfg);
  a.state = state; a.ctrl = ctrl; a.learn = 1; a.lr = *lr; a.hp = *hp; a.sample_out = sample_out;
  a.grad_norm_out = const_cast<float*>(&ctrl->grad_norm);
  if (replay) a.replay = *replay;
  if (out) a.out = *out;
  return launch_act<MODE_TICK>(a, n_tiles(cfg), (hipStream_t)stream);
}

int swarm_rollout(const swarm_config* cfg, const float* params, float* state, int32_t n_ticks, uint32_t tick0,
                  float eps, const swarm_act_out* out, void* stream) {
  if (int e = check_cfg(cfg)) return e;
  if (n_ticks < 0 || cfg->graph == SWARM_GRAPH_DENSE) return SWARM_E_BADARG;
  ActArgs a = make_args(cfg);
  a.params = params; a.state = state; a.n_ticks = n_ticks; a.tick0 = tick0; a.eps = eps;
  if (out) a.out = *out;
  if (n_ticks == 0) return 0;
  return launch_act<MODE_ROLLOUT>(a, n_tiles(cfg), (hipStream_t)stream);
}

#if SWARM_STAMPS
int swarm_dbg_stamps_act(void* p) { return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_swarm_stamps), &p, sizeof(p)); }
#endif

int swarm_host_topk_set(const float* dist, int32_t n, int32_t k, uint8_t* selected) {
  if (!dist || !selected || n < 1 || n > 32) return SWARM_E_BADARG;
  if (k < 1 || k > n) return SWARM_E_KNN_K;
  const uint32_t m = topk_smallest_mask<32>(dist, n, k);
  for (int j = 0; j < n; ++j) selected[j] = (uint8_t)((m >> j) & 1u);
  return 0;
}

}  // extern "C"
