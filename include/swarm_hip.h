/* swarm_hip.h — C ABI of libswarm_hip.so, the MI355X (gfx950) hot path of the
 * swarm-RL inner loop of davidedomini/experiments-2025-acsos-marl-for-swarming-behaviors.
 *
 * Conventions:
 *   - every buffer is caller-owned DEVICE memory, contiguous, fp32 / int32 / uint8;
 *   - `stream` is a hipStream_t passed as void* (0 = legacy default stream);
 *   - every entry point returns 0 on success, a positive hipError_t, or a
 *     negative SWARM_E_* code; nothing throws across the ABI;
 *   - no allocation, no host synchronisation inside any call: every call can be
 *     captured into a hipGraph (the one exception: the peer exchange's setup calls,
 *     swarm_peer_alloc / _free / _ipc_*, made once before any tick).
 *
 * Reference interfaces each entry point replaces are cited per function
 * (paths relative to the reference checkout; VMAS 1.4.0 / PyG 2.5.3 are the
 * reference's third-party dependencies, restated in SURVEY.md §8(a)).
 */
#ifndef SWARM_HIP_H
#define SWARM_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SWARM_ABI_VERSION 10

#define SWARM_E_BADARG (-1)    /* invalid shape / config */
#define SWARM_E_KNN_K (-2)     /* k > n_agents: torch.topk "selected index k out of range" */
#define SWARM_E_NOGPU (-3)
#define SWARM_E_UNSUPPORTED (-4) /* configuration has no fused-tick kernel (use the 3-launch tick) */

/* SWARM_FLOCKING: src/scenarios/flocking_scenario.py (the reference's third scenario class,
   train_gcn_dqn.py:244-245); needs n_agents >= 2 */
enum swarm_scenario { SWARM_GOTO = 0, SWARM_OBSTACLE_AVOIDANCE = 1, SWARM_FLOCKING = 2 };
enum swarm_graph { SWARM_GRAPH_COMPLETE = 0, SWARM_GRAPH_KNN = 1, SWARM_GRAPH_DENSE = 2, SWARM_GRAPH_RADIUS = 3 };
enum swarm_conv { SWARM_CONV_GAT = 0, SWARM_CONV_GCN = 1 };
/* Q-network: GCN = the reference's GCN class (one GATConv, hidden 32; params N_PARAMS = 1673;
   trainable).  GAT3 = the same class with its commented conv2/conv3 layers (train_gcn_dqn.py:54-55,
   65-68), hidden 8, 409 params: what data/models/experiment_Flocking-seed_*.pth hold.  GAT3 is
   forward only (swarm_q_forward, swarm_act_step, swarm_rollout); the learner entry points return
   SWARM_E_UNSUPPORTED for it. */
enum swarm_net { SWARM_NET_GCN = 0, SWARM_NET_GAT3 = 1 };
#define SWARM_GAT3_N_PARAMS 409

/* Static description of a batch of vectorised environments (one rank's shard). */
typedef struct swarm_config {
  int32_t n_envs;       /* B: environments handled by this call                         */
  int32_t n_agents;     /* N: agents per environment, 1..32                             */
  int32_t scenario;     /* swarm_scenario                                               */
  int32_t graph;        /* swarm_graph: complete (train_gcn_dqn.py:101-108), kNN (simulator.py:15-24),
                           DENSE = caller-supplied multiplicity matrix [B][N][N] uint8, or
                           RADIUS = radius-neighbour graph (north_star):
                           edge u -> v for u != v with |p_u - p_v| <= radius, plus (0, 0)  */
  int32_t knn_k;        /* k of the kNN graph (reference code: 10, recorded data: 5)    */
  int32_t conv;         /* swarm_conv: GAT (the reference's GCN class) or GCNConv (a13) */
  int32_t env_offset;   /* global index of env 0 (rank sharding; keys the RNG)          */
  int32_t flags;        /* SWARM_F_* bits                                               */
  uint64_t seed;        /* Philox key                                                   */
  float radius;         /* neighbour radius of SWARM_GRAPH_RADIUS (> 0)                 */
  int32_t net;          /* swarm_net (GAT3 requires conv == SWARM_CONV_GAT)             */
} swarm_config;

#define SWARM_F_SHARED_RESET 1   /* one reset centre for all envs (go_to_position_scenario.py:88) */
#define SWARM_F_RANDOM_OA 2      /* ObstacleAvoidance random=True (obstacle_avoidance_scenario.py:100) */

/* Device-resident control block; kernels read and advance it so that a tick
 * sequence can be replayed from a captured hipGraph.  Layout is ABI. */
typedef struct swarm_ctrl {
  uint32_t tick;          /* completed ticks (the reference's `ticks` is tick + 1 during a tick) */
  uint32_t write_slot;    /* replay slot the next tick writes                               */
  uint32_t filled_slots;  /* valid replay slots, <= capacity                                */
  uint32_t adam_step;     /* optimizer steps taken                                          */
  float eps;              /* exploration epsilon for the next tick                          */
  float loss;             /* last TD loss (0 when the update was skipped)                   */
  float grad_norm;        /* last pre-clip global gradient norm                             */
  uint32_t trained;       /* 1 = an optimizer step is pending (fused tick: applied by the next
                             swarm_train_act_step or by swarm_adam_flush); 0 after swarm_adam_step */
  uint32_t episode;       /* episode counter (reset RNG key)                                */
  uint32_t pad0;
  uint32_t beta_pow[4];   /* beta1^adam_step, beta2^adam_step as two little-endian doubles
                             (words 10-13)                                                  */
  float adam_step_size;   /* Adam scalars of optimizer step adam_step + 1, kept current by the */
  float adam_inv_bc2;     /* library: lr / (1 - beta1^(s+1)) and 1 / sqrt(1 - beta2^(s+1))     */
  uint32_t sample_key[4]; /* cache: replay-sampling round keys of tick `sample_tick` over      */
  uint32_t sample_tick;   /* `sample_n` graphs, prepared by swarm_reduce_advance (words 16-22); */
  uint32_t sample_n;      /* recomputed from (tick, n) whenever the tags do not match          */
  uint32_t sample_bits;
  uint32_t peer_hold;     /* word 23, sticky: 1 once a peer-exchange wait of swarm_reduce_advance_peer
                             expired on this rank; every later optimizer step is then skipped (the
                             summed gradient is wrong), so a timeout never reaches the weights.
                             Cleared only by swarm_ctrl_init; PeerExchange.check() raises on it. */
  float one_m_beta1;      /* words 24-25: (float)(1 - beta1), (float)(1 - beta2) formed in double from   */
  float one_m_beta2;      /* swarm_adam_cfg's double betas by swarm_ctrl_init, as torch forms them, and
                             rewritten by every swarm_reduce_advance[_peer]; swarm_adam_step / _flush
                             form them from their swarm_adam_cfg when a word is 0 (a control block
                             that skipped swarm_ctrl_init), so no step freezes m and v            */
  uint32_t pad1[6];
} swarm_ctrl;           /* 32 words */
/* A fresh control block comes from swarm_ctrl_init (all counters 0, beta powers 1). */

/* Replay ring (GraphReplayBuffer, train_gcn_dqn.py:25-48), SoA, per rank:
 * slot t holds the B transitions pushed at one tick. Graph id g = slot*B + env. */
typedef struct swarm_replay {
  float* s;          /* [cap][B][N][4]  state before the tick: pos.xy, vel.xy */
  float* s_next;     /* [cap][B][N][4]  state after the tick                 */
  float* r;          /* [cap][B][N]     per-agent reward                     */
  uint8_t* a;        /* [cap][B][N]     action                               */
  int32_t capacity;  /* slots                                                */
  int32_t pad;
} swarm_replay;

/* Per-tick outputs of the fused acting step; every pointer may be NULL. */
typedef struct swarm_act_out {
  float* q;          /* [B][N][9] Q-values                       */
  int32_t* actions;  /* [B][N] chosen actions                    */
  float* reward;     /* [B][N]                                   */
  float* obs;        /* [B][N][6] pos, vel, goal after the step  */
  float* avg_dist;   /* [B] scenario.average_distance_to_goal()  */
  float* hits;       /* [B] scenario.obstacles_hits()            */
  uint8_t* mult;     /* [B][N][N] edge multiplicity used         */
  float* traj_pos;   /* rollout only: [T][B][N][2] positions after every tick */
  float* traj_dist;  /* rollout only: [T][B] avg distance to goal per tick    */
  float* traj_hits;  /* rollout only: [T][B] obstacle hits per tick          */
} swarm_act_out;

/* Optimizer hyper-parameters (train_gcn_dqn.py:85,112-137). */
typedef struct swarm_adam_cfg {
  float lr, beta1, beta2, eps;   /* Adam(lr=1e-3), torch defaults                 */
  float max_norm;                /* clip_grad_norm_(…, 1)                          */
  float gamma;                   /* 0.99                                           */
  int32_t batch;                 /* sampled graphs per update (reference 32)       */
  int32_t update_target_every;   /* 200 at train_gcn_dqn.py:175                   */
  int32_t world_size;            /* ranks whose gradients are summed (grad /= W)   */
  int32_t flags;                 /* SWARM_ADAM_F_* (ABI 10; was padding)           */
  /* the same lr / betas in double, as torch.optim.Adam holds them (Python floats): 1 - beta
     (into the control block by swarm_ctrl_init) and the bias corrections are formed from these
     as torch forms them (ABI 9); 0 = use the float fields */
  double lr_d, beta1_d, beta2_d;
} swarm_adam_cfg;

/* swarm_adam_cfg.flags.  SWARM_ADAM_F_NORM_PARTIALS: the clip norm's group partials in lr->grad
 * (SWARM_GRAD_SQ_BASE, written by the slab reduce) belong to lr->grad as it is: the launch's
 * optimizer step then reads those 105 values instead of reducing the whole gradient behind a
 * block barrier (swarm_train_tick, swarm_train_act_step).  Set it when nothing changed lr->grad
 * after swarm_reduce_advance / _peer (one rank, or the fused peer exchange); clear it when an
 * all-reduce of the gradient (RCCL) or a caller wrote lr->grad in between.  Both ways give the
 * same bits: the partials are the same fixed-order sums the step forms otherwise. */
#define SWARM_ADAM_F_NORM_PARTIALS 1

/* Gradient buffers (swarm_learner.grad, the grad of swarm_grad_reduce / swarm_adam_step) hold
 * SWARM_GRAD_FLOATS floats: [0, N_PARAMS) the gradient, [N_PARAMS] the sum of squared TD errors,
 * then at SWARM_GRAD_SQ_BASE the clip norm's 105 group partials the slab reduce writes beside the
 * gradient (ABI 10): partial j = (d[4j] + d[4j+1]) + (d[4j+2] + d[4j+3]) over the float4 groups
 * d[i] = ((g0^2 + g1^2) + g2^2) + g3^2 of parameters 4i..4i+3 (each g scaled by 1/world_size when
 * world_size > 1; parameters >= N_PARAMS count 0); the squared norm is then
 * wave_sum(partial[l] + partial[l + 64]) over lanes l = 0..63 (swarm_adam.h). */
#define SWARM_GRAD_SQ_BASE 1680
#define SWARM_GRAD_SQ_COUNT 105
#define SWARM_GRAD_FLOATS 1792

/* Learner state for the fused training tick.  Weights/moments are ping-ponged so
 * that every block of swarm_train_act_step can read the previous tick's values
 * while block 0 persists the new ones: tick t reads *_cur, writes *_nxt;
 * swarm_reduce_advance copies *_nxt back to *_cur.  All buffers hold N_PARAMS
 * floats (grad: SWARM_GRAD_FLOATS, see above). */
typedef struct swarm_learner {
  float* w_cur;
  float* w_nxt;
  float* m_cur;
  float* m_nxt;
  float* v_cur;
  float* v_nxt;
  float* target;
  float* grad;
} swarm_learner;

int swarm_abi_version(void);
int swarm_n_params(void);                 /* 1673 */
const char* swarm_build_info(void);

/* Environment state: [B][N][4] floats (pos.xy, vel.xy) for every scenario.  SWARM_FLOCKING
 * keeps per-agent scenario state after it: [B][N] floats of previous_distance_to_agents
 * (flocking_scenario.py:110-122 at reset, :163-164 per reward call), which every entry point
 * that steps the env reads and writes.  swarm_state_floats gives the buffer size. */
int64_t swarm_state_floats(const swarm_config* cfg);

/* Reset: reset_world_at + generate_grid (go_to_position_scenario.py:52-106,
 * obstacle_avoidance_scenario.py:63-133, flocking_scenario.py:86-122) for all B envs. */
int swarm_env_reset(const swarm_config* cfg, float* state, uint32_t episode, void* stream);

/* Recompute the scenario state that follows [B][N][4] (Flocking; a no-op otherwise) from the
 * positions in `state`, after a caller wrote them: fresh != 0 as reset_world_at leaves it (the
 * reset loop measures agent i against the new positions of agents < i and the zeroed ones of
 * agents > i, flocking_scenario.py:93-122), fresh == 0 as a step's reward call leaves it. */
int swarm_env_sync_state(const swarm_config* cfg, float* state, int32_t fresh, void* stream);

/* VMAS Environment.step for discrete actions (call sites train_gcn_dqn.py:169,
 * simulator.py:68): decode, holonomic force, sphere collisions, drag/Euler,
 * scenario reward/observation/metrics.  actions [B][N] int32. */
int swarm_env_step(const swarm_config* cfg, float* state, const int32_t* actions,
                   const swarm_act_out* out, void* stream);

/* Graph build: DQNTrainer.create_graph_from_observations (train_gcn_dqn.py:94-110)
 * and simulator.create_graph_from_observations (simulator.py:9-26) as a dense
 * per-env edge multiplicity mult[b][u][v] = #edges u->v.  pos from x[:, :2]. */
int swarm_build_graph(const swarm_config* cfg, const float* x, uint8_t* mult, void* stream);

/* PyG edge_index [2][E] int64 of a Batch of n_graphs graphs with n_nodes nodes each
 * (Batch.from_data_list, train_gcn_dqn.py:45) -> dense multiplicity [G][N][N] uint8.
 * mult must be 4-byte aligned with room for roundup4(G*N*N) bytes; *err (device
 * int32) is set to 1 if an edge leaves its graph.  Multiplicities must stay < 256. */
int swarm_edges_to_mult(const int64_t* edge_index, int64_t n_edges, int32_t n_graphs,
                        int32_t n_nodes, uint8_t* mult, int32_t* err, void* stream);

/* GCN.forward (train_gcn_dqn.py:59-70) on B per-env graphs of N nodes.
 * x [B*N][7] node features; mult NULL unless cfg->graph == SWARM_GRAPH_DENSE. */
int swarm_q_forward(const swarm_config* cfg, const float* params, const float* x,
                    const uint8_t* mult, float* q, void* stream);

/* Fused acting tick (train_gcn_dqn.py:161-172 / simulator.py:59-68):
 * graph -> GAT Q -> eps-greedy (ctrl->eps, Philox) -> env.step -> replay push
 * (replay may be NULL).  state updated in place. */
int swarm_act_step(const swarm_config* cfg, const float* params, float* state,
                   const swarm_replay* replay, const swarm_ctrl* ctrl,
                   const swarm_act_out* out, void* stream);

/* Fused training tick, acting half (train_gcn_dqn.py:161-172 + the optimizer step
 * of the previous tick's TD loss, :125-133): if ctrl->trained, apply
 * clip_grad_norm_ + Adam to (w_cur, grad) in every block (LDS image), block 0
 * persists w_nxt/m_nxt/v_nxt (+ target sync); then act with w_nxt.  If sample_out
 * != NULL it also draws this tick's TD batch indices [hp->batch] (exactly what
 * swarm_td_grad would draw in-kernel; pass them to it as sample_in).
 * Sequence per tick: swarm_train_act_step -> swarm_td_grad(params = w_nxt) ->
 * swarm_reduce_advance [-> all-reduce(grad)]. */
int swarm_train_act_step(const swarm_config* cfg, const swarm_adam_cfg* hp, const swarm_learner* lr,
                         float* state, const swarm_replay* replay, const swarm_ctrl* ctrl,
                         const swarm_act_out* out, int32_t* sample_out, void* stream);

/* Fused training tick in ONE launch (train_gcn_dqn.py:153-178 without the optimizer's
 * launch): acting blocks (as swarm_train_act_step) and TD blocks (as swarm_td_grad with
 * in-kernel sampling) run side by side; both apply the pending optimizer step in registers.
 * TD graphs drawn from this tick's replay slot (the reference pushes before it samples,
 * :170-172) read the acting waves' write-through hand-off records in `workspace`
 * (swarm_train_tick_workspace_bytes; zero it whenever ctrl is (re)initialised).  Follow with
 * swarm_reduce_advance [-> all-reduce(grad)].  Bit-identical to the 3-launch sequence.
 * Complete, kNN or radius training graph, GAT or GCNConv, n_agents <= 16; else SWARM_E_UNSUPPORTED. */
int swarm_train_tick_supported(const swarm_config* cfg);
int64_t swarm_train_tick_workspace_bytes(const swarm_config* cfg);
int swarm_train_tick(const swarm_config* cfg, const swarm_adam_cfg* hp, const swarm_learner* lr, float* state,
                     const swarm_replay* replay, const swarm_ctrl* ctrl, const swarm_act_out* out,
                     float* slabs, void* workspace, int32_t* sample_out, void* stream);

/* Host reference of the replay-batch permutation (GraphReplayBuffer.sample restated as a
 * keyed Feistel permutation; tests): index = batch position -> graph id, and its inverse. */
uint32_t swarm_host_sample_index(uint32_t i, uint32_t n, uint32_t k0, uint32_t k1, uint32_t tick);
uint32_t swarm_host_sample_position(uint32_t g, uint32_t n, uint32_t k0, uint32_t k1, uint32_t tick);

/* Slab sum -> lr->grad, copy *_nxt -> *_cur, record the pending update and
 * advance ctrl (tick, replay slot, the next step's Adam scalars). */
int swarm_reduce_advance(const swarm_config* cfg, const swarm_adam_cfg* hp, const float* slabs,
                         const swarm_learner* lr, int32_t replay_capacity, swarm_ctrl* ctrl, void* stream);

/* ---- Peer all-reduce over xGMI (the one exchange of the data-parallel tick).
 * The reference has no distributed code; this replaces the RCCL all_reduce(grad) that would
 * follow swarm_reduce_advance (dist.py allreduce_grad_).  Every rank owns one exchange buffer
 * (swarm_peer_alloc: uncached device memory, so a peer's xGMI stores are seen by this GPU's
 * loads without a cache flush) and maps every other rank's buffer through HIP IPC.  A rank
 * publishes each gradient column as a tagged 8-byte granule {tag, value} with ONE system-scope
 * store into every rank's buffer (its own included) and polls its own buffer until all W tags
 * match: the data is its own flag.  The W values of a column are added in rank order, so every
 * rank computes bitwise the same sum.  Tags come from per-block launch counters (`seq`, device
 * words zeroed once at setup; every rank must issue the same sequence of peer calls) and the
 * buffer is double-buffered by their parity, so nothing is ever reset.  Waits are bounded in
 * time: one that expires adds 1 to *err (the sum is then wrong: check err and fail loudly); in
 * swarm_reduce_advance_peer it also sets ctrl->peer_hold, which stops every later optimizer step
 * of this rank before it can apply the wrong sum. */
#define SWARM_PEER_MAX 8
#define SWARM_PEER_HANDLE_BYTES 64   /* hipIpcMemHandle_t */
#define SWARM_PEER_SEQ_WORDS 256     /* launch counters per rank (device uint32, zeroed at setup) */
typedef struct swarm_peer {
  int32_t world_size;              /* W, 1..SWARM_PEER_MAX                                     */
  int32_t rank;                    /* this rank                                                */
  void* recv[SWARM_PEER_MAX];      /* rank q's exchange buffer as mapped in this process       */
  uint32_t* seq;                   /* SWARM_PEER_SEQ_WORDS launch counters of this rank        */
  int32_t* err;                    /* device int32: waits that hit the time bound              */
  uint32_t timeout_us;             /* bound of one wait (0 = 5 000 000 us: ranks start skewed) */
  int32_t pad;
} swarm_peer;

/* Setup (host-synchronous, not for the hot path): bytes of one exchange buffer; allocate one
 * (zeroed, uncached) / free it; export its IPC handle (SWARM_PEER_HANDLE_BYTES bytes); map a
 * peer's handle / unmap it. */
int64_t swarm_peer_buffer_bytes(void);
int swarm_peer_alloc(void** buf);
int swarm_peer_free(void* buf);
int swarm_peer_ipc_handle(void* buf, void* handle);
int swarm_peer_ipc_open(const void* handle, void** buf);
int swarm_peer_ipc_close(void* buf);

/* swarm_reduce_advance with the all-reduce fused in: each column block sums its slab columns,
 * exchanges them with the other ranks and writes lr->grad = the rank-ordered sum over ranks
 * (ctrl->loss stays this rank's own loss, as with swarm_reduce_advance + RCCL). */
int swarm_reduce_advance_peer(const swarm_config* cfg, const swarm_adam_cfg* hp, const float* slabs,
                              const swarm_learner* lr, int32_t replay_capacity, swarm_ctrl* ctrl,
                              const swarm_peer* peer, void* stream);

/* Standalone in-place SUM all-reduce of x[n] (n <= N_PARAMS + 1) over the ranks of `peer`
 * (rank-ordered, bitwise identical on every rank); the unfused API path's replacement of
 * all_reduce(grad), and the setup self-test. */
int swarm_peer_allreduce(const swarm_peer* peer, float* x, int32_t n, void* stream);

/* Draw the TD batch's replay indices [batch] for the tick ctrl describes
 * (GraphReplayBuffer.sample, train_gcn_dqn.py:40: keyed permutation, distinct ids). */
int swarm_sample_prepare(const swarm_config* cfg, const swarm_adam_cfg* hp, int32_t replay_capacity,
                         const swarm_ctrl* ctrl, int32_t* samples, void* stream);

/* Apply a pending update (ctrl->trained) to w_cur/m_cur/v_cur in place, e.g. after
 * the last fused tick.  No tick advance. */
int swarm_adam_flush(const swarm_config* cfg, const swarm_adam_cfg* hp, const swarm_learner* lr,
                     swarm_ctrl* ctrl, void* stream);

/* Acting-only rollout of n_ticks ticks with frozen weights in ONE launch
 * (Simulator.run_simulation, simulator.py:59-93, greedy when eps = 0).
 * out->reward / avg_dist / hits accumulate per-env sums over the ticks. */
int swarm_rollout(const swarm_config* cfg, const float* params, float* state,
                  int32_t n_ticks, uint32_t tick0, float eps, const swarm_act_out* out, void* stream);

/* Workspace (floats) of swarm_td_grad's per-block gradient slabs. */
int64_t swarm_td_workspace_floats(const swarm_config* cfg, int32_t batch);

/* DQN TD-loss gradient (train_gcn_dqn.py:113-124): sample `batch` graphs from the
 * replay (keyed Philox permutation; or sample_in [batch] graph ids if non-NULL),
 * online forward, target forward + max, MSE, backward.  Writes per-block
 * gradient slabs (+ loss partial in column N_PARAMS) to `slabs`.
 * Skips (zero slabs, ctrl unchanged) while the replay holds < batch graphs. */
int swarm_td_grad(const swarm_config* cfg, const swarm_adam_cfg* hp, const float* params,
                  const float* target, const swarm_replay* replay, const swarm_ctrl* ctrl,
                  const int32_t* sample_in, int32_t* sample_out, float* slabs, void* stream);

/* Deterministic fixed-order sum of the slabs -> grad[N_PARAMS + 1] (last = loss sum), plus the
 * clip norm's group partials at SWARM_GRAD_SQ_BASE (grad holds SWARM_GRAD_FLOATS floats). */
int swarm_grad_reduce(const swarm_config* cfg, const swarm_adam_cfg* hp, const float* slabs,
                      float* grad, void* stream);

/* clip_grad_norm_(1) + Adam step + target sync every `update_target_every` ticks,
 * then advance ctrl (tick, replay slot).  grad is the (all-reduced) gradient sum. */
int swarm_adam_step(const swarm_config* cfg, const swarm_adam_cfg* hp, float* params,
                    float* target, float* adam_m, float* adam_v, const float* grad,
                    int32_t replay_capacity, swarm_ctrl* ctrl, void* stream);

/* Initialise a control block: counters 0, eps, beta^0 = 1 and the Adam scalars of step 1. */
int swarm_ctrl_init(const swarm_adam_cfg* hp, float eps, swarm_ctrl* ctrl, void* stream);

/* Advance ctrl after an acting-only tick (no optimizer). */
int swarm_ctrl_advance(const swarm_config* cfg, const swarm_replay* replay, swarm_ctrl* ctrl, void* stream);

/* Host reference of the per-row neighbour selection the kernels run (CPU
 * torch.topk(largest=False) set semantics, libstdc++ introselect); for tests. */
int swarm_host_topk_set(const float* dist, int32_t n, int32_t k, uint8_t* selected);

#ifdef __cplusplus
}
#endif
#endif /* SWARM_HIP_H */
