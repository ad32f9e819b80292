"""SwarmEngine: one rank's shard of vectorised swarm environments plus the DQN learner,
all resident in HBM, driven through libswarm_hip.so.

One fused training tick (the reference's hot loop, src/training/train_gcn_dqn.py:153-178):

    swarm_train_tick      acting blocks: [clip + Adam of the previous tick's gradient, target
                          sync] graph -> GAT Q -> eps-greedy -> env.step -> replay push;
                          TD blocks beside them: [the same optimizer step] batch rows ->
                          target fwd -> online fwd -> TD loss -> backward              (1 launch)
    swarm_reduce_advance  deterministic slab sum, ping-pong copy-back, ctrl advance    (1 launch)
    [all_reduce(grad) over RCCL when world_size > 1]

With a ``PeerExchange`` (dist.py; ``peer=``) the all-reduce is fused into the reduce launch
(``swarm_reduce_advance_peer``: xGMI stores of the column sums, rank-ordered sum): still two
launches per tick at any world size, and no collective in the captured graph.

TD graphs drawn from the tick's own replay slot (push before sample, as the reference)
wait in-kernel for the acting wave of their env (write-through hand-off records in
``tick_ws``).  Configurations without a fused-tick kernel (kNN training graph,
n_agents > 16) run the 3-launch tick (``train_tick3``: swarm_train_act_step ->
swarm_td_grad -> swarm_reduce_advance); both are bit-identical to each other and to the
unfused API sequence.

The optimizer step of tick t runs at the start of tick t+1's acting launch (before any
use of the weights), so every weight the reference would use is used; ``flush()``
applies the last pending step.  The unfused sequence (``act`` + ``td_update``:
act / td_grad / grad_reduce / adam_step) is kept for API calls and as the parity
reference of the fused one (bit-identical, tests/test_gpu_parity.py).

Every launch goes to torch's current stream, so a run of ticks can be captured
once into a hipGraph (``capture``) and replayed.  There is no CPU fallback.
"""
from __future__ import annotations

import math
from typing import Optional

import torch

from . import _lib
from .dist import allreduce_grad_
from ._lib import (CTRL, N_PARAMS, SwarmActOut, SwarmAdamCfg, SwarmConfig, SwarmLearner, SwarmReplay, check, ptr,
                   stream_ptr)

SCENARIOS = {"GoTo": _lib.SWARM_GOTO, "ObstacleAvoidance": _lib.SWARM_OBSTACLE_AVOIDANCE,
             "Flocking": _lib.SWARM_FLOCKING, "go_to": _lib.SWARM_GOTO,
             "obstacle_avoidance": _lib.SWARM_OBSTACLE_AVOIDANCE, "flocking": _lib.SWARM_FLOCKING}
GRAPHS = {"complete": _lib.GRAPH_COMPLETE, "knn": _lib.GRAPH_KNN, "radius": _lib.GRAPH_RADIUS}
CONVS = {"gat": _lib.CONV_GAT, "gcn": _lib.CONV_GCN}
NETS = {"gcn": _lib.NET_GCN, "gat3": _lib.NET_GAT3}

PARAM_ORDER = (
    ("conv1.att_src", (1, 1, 32)), ("conv1.att_dst", (1, 1, 32)), ("conv1.bias", (32,)),
    ("conv1.lin.weight", (32, 7)), ("lin1.weight", (32, 32)), ("lin1.bias", (32,)),
    ("lin2.weight", (9, 32)), ("lin2.bias", (9,)),
)

# the three-layer GAT of the Flocking checkpoints (data/models/experiment_Flocking-seed_*.pth;
# the GCN class with its commented conv2/conv3, train_gcn_dqn.py:54-55,65-68), hidden 8
PARAM_ORDER_GAT3 = tuple(
    (f"conv{i}.{n}", s) for i, k in ((1, 7), (2, 8), (3, 8))
    for n, s in (("att_src", (1, 1, 8)), ("att_dst", (1, 1, 8)), ("bias", (8,)), ("lin.weight", (8, k))))
PARAM_ORDER_GAT3 += (("lin1.weight", (8, 8)), ("lin1.bias", (8,)), ("lin2.weight", (9, 8)), ("lin2.bias", (9,)))


def param_order(net: str = "gcn"):
    return PARAM_ORDER_GAT3 if net == "gat3" else PARAM_ORDER


def flatten_state_dict(sd, device=None, net: str = "gcn") -> torch.Tensor:
    return torch.cat([sd[k].detach().reshape(-1).to(torch.float32) for k, _ in param_order(net)]).to(device)


def unflatten_params(flat: torch.Tensor, net: str = "gcn") -> dict:
    out, o = {}, 0
    for k, shape in param_order(net):
        n = math.prod(shape)
        out[k] = flat[o:o + n].reshape(shape).clone()
        o += n
    return out


def glorot_init(generator: torch.Generator) -> torch.Tensor:
    """Fresh GCN parameters: glorot for GATConv weights/attention (PyG reset_parameters),
    torch.nn.Linear default init for lin1/lin2, zero GAT bias.  Init is not pinned by
    any reference artefact; training runs normally start from it."""
    def glorot(shape, fan_in, fan_out):
        a = math.sqrt(6.0 / (fan_in + fan_out))
        return (torch.rand(shape, generator=generator) * 2 - 1) * a

    def linear(out_f, in_f):
        b = 1.0 / math.sqrt(in_f)
        w = (torch.rand(out_f, in_f, generator=generator) * 2 - 1) * b
        bias = (torch.rand(out_f, generator=generator) * 2 - 1) * b
        return w, bias

    sd = {
        "conv1.att_src": glorot((1, 1, 32), 1, 32),
        "conv1.att_dst": glorot((1, 1, 32), 1, 32),
        "conv1.bias": torch.zeros(32),
        "conv1.lin.weight": glorot((32, 7), 7, 32),
    }
    sd["lin1.weight"], sd["lin1.bias"] = linear(32, 32)
    sd["lin2.weight"], sd["lin2.bias"] = linear(9, 32)
    return flatten_state_dict(sd)


class SwarmEngine:
    def __init__(self, scenario="GoTo", n_agents: int = 8, n_envs: int = 1024, *, seed: int = 0,
                 graph: str = "complete", knn_k: int = 10, conv: str = "gat", params=None, radius: float = 0.3,
                 batch: Optional[int] = None, gamma: float = 0.99, lr: float = 1e-3, betas=(0.9, 0.999),
                 adam_eps: float = 1e-8, max_norm: float = 1.0, update_target_every: int = 200,
                 replay_capacity: int = 1_000_000, env_offset: int = 0, world_size: int = 1,
                 process_group=None, shared_reset: bool = False, random_oa: bool = True, eps: float = 0.05,
                 device=None, learn: bool = True, net: str = "gcn", peer=None):
        self.lib = _lib.load()
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        if self.device.type != "cuda":
            raise RuntimeError("SwarmEngine runs on a ROCm GPU only (no CPU fallback)")
        sid = SCENARIOS[scenario] if isinstance(scenario, str) else int(scenario)
        flags = (_lib.F_SHARED_RESET if shared_reset else 0) | (_lib.F_RANDOM_OA if random_oa else 0)
        if net == "gat3" and learn:
            raise ValueError("net='gat3' (the Flocking checkpoints' three-layer GAT) is forward only: use learn=False")
        self.net = net
        self.cfg = SwarmConfig(n_envs, n_agents, sid, GRAPHS[graph], knn_k, CONVS[conv], env_offset, flags,
                               seed & 0xFFFFFFFFFFFFFFFF, float(radius), NETS[net])
        self.B, self.N = n_envs, n_agents
        self.scenario_id = sid
        self.batch = n_envs if batch is None else batch
        self.world_size = world_size
        self.process_group = process_group
        if peer is not None and peer.world_size != world_size:
            raise ValueError(f"peer exchange of {peer.world_size} ranks for world_size {world_size}")
        self.peer = peer
        # the double fields: torch.optim.Adam's Python-float lr / betas (1 - beta, bias corrections)
        self.hp = SwarmAdamCfg(lr, betas[0], betas[1], adam_eps, max_norm, gamma, self.batch,
                               update_target_every, world_size, 0, float(lr), float(betas[0]), float(betas[1]))
        dev = self.device
        f32 = dict(dtype=torch.float32, device=dev)
        # [B][N][4] pos.xy, vel.xy; Flocking keeps its per-agent previous_distance_to_agents after
        # it (swarm_state_floats), as `scenario_state` [B][N]
        nst = int(self.lib.swarm_state_floats(ctypes_ref(self.cfg)))
        check(min(nst, 0), "swarm_state_floats")
        self._state_buf = torch.zeros(max(nst, 1), **f32)
        self.state = self._state_buf[: n_envs * n_agents * 4].view(n_envs, n_agents, 4)
        self.scenario_state = (self._state_buf[n_envs * n_agents * 4: nst].view(n_envs, n_agents)
                               if nst > n_envs * n_agents * 4 else None)
        n_par = _lib.GAT3_N_PARAMS if net == "gat3" else N_PARAMS
        if params is None:
            if net == "gat3":
                raise ValueError("net='gat3' needs params (a Flocking checkpoint)")
            g = torch.Generator().manual_seed(seed)
            params = glorot_init(g)
        elif isinstance(params, dict):
            params = flatten_state_dict(params, net=net)
        p0 = params.detach().to(**f32).reshape(-1)
        assert p0.numel() == n_par
        # learner buffers: [w_cur, w_nxt, m_cur, m_nxt, v_cur, v_nxt, target] rows + grad
        self._lrn = torch.zeros(7, N_PARAMS + 3, **f32)       # +3: rows stay 16-B aligned
        self.params, self.w_nxt = self._lrn[0, :n_par], self._lrn[1, :n_par]
        self.adam_m, self.m_nxt = self._lrn[2, :n_par], self._lrn[3, :n_par]
        self.adam_v, self.v_nxt = self._lrn[4, :n_par], self._lrn[5, :n_par]
        self.target = self._lrn[6, :n_par]
        self.params.copy_(p0)
        self.target.copy_(p0)
        self.ctrl = torch.zeros(_lib.CTRL_WORDS, dtype=torch.int32, device=dev)
        check(self.lib.swarm_ctrl_init(ctypes_ref(self.hp), float(eps), ptr(self.ctrl), stream_ptr()),
              "swarm_ctrl_init")
        self.episode = 0
        cap = max(1, -(-replay_capacity // n_envs)) if learn else 1
        self.capacity = cap
        self.rep_s = torch.zeros(cap, n_envs, n_agents, 4, **f32)
        self.rep_s1 = torch.zeros(cap, n_envs, n_agents, 4, **f32)
        self.rep_r = torch.zeros(cap, n_envs, n_agents, **f32)
        self.rep_a = torch.zeros(cap, n_envs, n_agents, dtype=torch.uint8, device=dev)
        self.replay = SwarmReplay(ptr(self.rep_s), ptr(self.rep_s1), ptr(self.rep_r), ptr(self.rep_a), cap, 0)
        ws = self.lib.swarm_td_workspace_floats(ctypes_ref(self.cfg), self.batch) if net == "gcn" else 4
        if ws < 0:
            check(int(ws), "swarm_td_workspace_floats")
        self.fused = learn and bool(self.lib.swarm_train_tick_supported(ctypes_ref(self.cfg)))
        self.slabs = torch.zeros(int(ws), **f32)
        # + the reduce's norm partials (ABI 10); a write to grad from outside the library's reduce
        # must be declared with grad_written() (the partials then no longer describe it)
        self.grad = torch.zeros(_lib.GRAD_FLOATS, **f32)
        self._grad_dirty = False
        self.learner = SwarmLearner(*[ptr(self._lrn[i]) for i in range(7)], ptr(self.grad))
        self.samples = torch.zeros(max(self.batch, 1), dtype=torch.int32, device=dev)
        # fused-tick workspace (error word, launch counters, hand-off granule records); zeroed with ctrl
        self.tick_ws = None
        if self.fused:
            nb = self.lib.swarm_train_tick_workspace_bytes(ctypes_ref(self.cfg))
            check(int(min(nb, 0)), "swarm_train_tick_workspace_bytes")
            self.tick_ws = torch.zeros(int(nb), dtype=torch.uint8, device=dev)
        # per-tick outputs
        self.q = torch.zeros(n_envs, n_agents, 9, **f32)
        self.actions = torch.zeros(n_envs, n_agents, dtype=torch.int32, device=dev)
        self.reward = torch.zeros(n_envs, n_agents, **f32)
        self.obs = torch.zeros(n_envs, n_agents, 6, **f32)
        self.avg_dist = torch.zeros(n_envs, **f32)
        self.hits = torch.zeros(n_envs, **f32)
        self.out = SwarmActOut(ptr(self.q), ptr(self.actions), ptr(self.reward), ptr(self.obs),
                               ptr(self.avg_dist), ptr(self.hits), 0, 0, 0, 0)
        self.out_min = SwarmActOut(0, 0, ptr(self.reward), 0, ptr(self.avg_dist), ptr(self.hits), 0, 0, 0, 0)

    # ------------------------------------------------------------------ control block
    def set_eps(self, eps: float):
        self.ctrl.view(torch.float32)[CTRL["eps"]].fill_(float(eps))

    def read_ctrl(self) -> dict:
        c = self.ctrl.cpu()
        f = c.view(torch.float32)
        return dict(tick=int(c[0]), write_slot=int(c[1]), filled_slots=int(c[2]), adam_step=int(c[3]),
                    eps=float(f[4]), loss=float(f[5]), grad_norm=float(f[6]), trained=int(c[7]))

    def replay_len(self) -> int:
        """len(GraphReplayBuffer) in graphs (one graph = one env transition)."""
        return self.read_ctrl()["filled_slots"] * self.B

    # ------------------------------------------------------------------ env
    def reset(self, episode: Optional[int] = None):
        ep = self.episode if episode is None else episode
        check(self.lib.swarm_env_reset(ctypes_ref(self.cfg), ptr(self.state), ep, stream_ptr()), "swarm_env_reset")
        self.episode = ep + 1
        return self.state

    def set_state(self, pos: torch.Tensor, vel: torch.Tensor, fresh: bool = False):
        """Write agent positions/velocities [B, N, 2] and bring the scenario's per-agent state in
        line with them (Flocking): fresh=True as right after reset_world_at, else as after a step."""
        self.state.copy_(torch.cat([pos, vel], -1).to(self.state))
        check(self.lib.swarm_env_sync_state(ctypes_ref(self.cfg), ptr(self.state), int(fresh), stream_ptr()),
              "swarm_env_sync_state")

    def env_step(self, actions: torch.Tensor, out: Optional[SwarmActOut] = None):
        a = actions.to(device=self.device, dtype=torch.int32).contiguous()
        check(self.lib.swarm_env_step(ctypes_ref(self.cfg), ptr(self.state), ptr(a),
                                      ctypes_ref(out or self.out), stream_ptr()), "swarm_env_step")

    # ------------------------------------------------------------------ acting
    def act(self, push: bool = True, full_out: bool = True):
        check(self.lib.swarm_act_step(ctypes_ref(self.cfg), ptr(self.params), ptr(self.state),
                                      ctypes_ref(self.replay) if push else None, ptr(self.ctrl),
                                      ctypes_ref(self.out if full_out else self.out_min), stream_ptr()),
              "swarm_act_step")

    def advance(self):
        check(self.lib.swarm_ctrl_advance(ctypes_ref(self.cfg), ctypes_ref(self.replay), ptr(self.ctrl),
                                          stream_ptr()), "swarm_ctrl_advance")

    def rollout(self, n_ticks: int, tick0: int = 0, eps: float = 0.0, traj: bool = False, params=None):
        """Acting-only rollout in one launch.  Returns per-env sums (and per-tick
        trajectories when traj=True)."""
        dev = self.device
        res = dict(reward=torch.zeros(self.B, self.N, device=dev), hits=torch.zeros(self.B, device=dev),
                   avg_dist=torch.zeros(self.B, device=dev), obs=torch.zeros(self.B, self.N, 6, device=dev))
        if traj:
            res["traj_pos"] = torch.zeros(n_ticks, self.B, self.N, 2, device=dev)
            res["traj_dist"] = torch.zeros(n_ticks, self.B, device=dev)
            res["traj_hits"] = torch.zeros(n_ticks, self.B, device=dev)
        out = SwarmActOut(0, 0, ptr(res["reward"]), ptr(res["obs"]), ptr(res["avg_dist"]), ptr(res["hits"]), 0,
                          ptr(res.get("traj_pos")), ptr(res.get("traj_dist")), ptr(res.get("traj_hits")))
        p = self.params if params is None else params
        check(self.lib.swarm_rollout(ctypes_ref(self.cfg), ptr(p), ptr(self.state), n_ticks, tick0, eps,
                                     ctypes_ref(out), stream_ptr()), "swarm_rollout")
        return res

    # ------------------------------------------------------------------ learning
    def td_grad(self, sample_in: Optional[torch.Tensor] = None, sample_out: Optional[torch.Tensor] = None):
        check(self.lib.swarm_td_grad(ctypes_ref(self.cfg), ctypes_ref(self.hp), ptr(self.params), ptr(self.target),
                                     ctypes_ref(self.replay), ptr(self.ctrl), ptr(sample_in), ptr(sample_out),
                                     ptr(self.slabs), stream_ptr()), "swarm_td_grad")
        self._grad_dirty = False
        check(self.lib.swarm_grad_reduce(ctypes_ref(self.cfg), ctypes_ref(self.hp), ptr(self.slabs),
                                         ptr(self.grad), stream_ptr()), "swarm_grad_reduce")

    def _sync_flags(self):
        """swarm_adam_cfg.flags for the next launches: the reduce's clip-norm partials describe
        lr->grad only while nothing else has written it since the reduce that formed them: not
        after an all-reduce of the gradient (RCCL / gloo / by hand at W > 1), and not after a
        write declared with ``grad_written()``.  Otherwise the optimizer prologue forms
        the norm from the gradient itself (the same summation order, so both give the same bits)."""
        exact = (self.world_size == 1 or self.peer is not None) and not self._grad_dirty
        self.hp.flags = _lib.ADAM_F_NORM_PARTIALS if exact else 0

    def grad_written(self):
        """Declare a write to ``grad`` made outside the library's reduce (e.g. a hand-made
        all-reduce or a test's injected gradient): the next optimizer step then forms the clip
        norm from ``grad`` instead of the reduce's partials, which describe the overwritten
        values.  The next reduce launch (swarm_reduce_advance / swarm_grad_reduce) clears it."""
        self._grad_dirty = True

    def allreduce_grad(self):
        g = self.grad[:N_PARAMS + 1]   # parameters + loss sum (not the norm partials)
        allreduce_grad_(g, self.world_size, self.process_group, self.peer)

    def adam(self):
        check(self.lib.swarm_adam_step(ctypes_ref(self.cfg), ctypes_ref(self.hp), ptr(self.params), ptr(self.target),
                                       ptr(self.adam_m), ptr(self.adam_v), ptr(self.grad), self.capacity,
                                       ptr(self.ctrl), stream_ptr()), "swarm_adam_step")

    def flush(self):
        """Apply a pending fused optimizer step to the current weights (no-op if none)."""
        check(self.lib.swarm_adam_flush(ctypes_ref(self.cfg), ctypes_ref(self.hp), ctypes_ref(self.learner),
                                        ptr(self.ctrl), stream_ptr()), "swarm_adam_flush")

    def td_update(self, sample_in=None, sample_out=None):
        """Unfused TD update (API path): applies the optimizer step immediately."""
        self.flush()
        self.td_grad(sample_in, sample_out)
        self.allreduce_grad()
        self.adam()

    def train_tick_unfused(self, full_out: bool = False):
        self.act(push=True, full_out=full_out)
        self.td_update()

    # single launches of the fused tick (bench.py times each kernel as a back-to-back chain)
    def launch_train_act(self):
        self._sync_flags()
        check(self.lib.swarm_train_act_step(ctypes_ref(self.cfg), ctypes_ref(self.hp), ctypes_ref(self.learner),
                                            ptr(self.state), ctypes_ref(self.replay), ptr(self.ctrl),
                                            ctypes_ref(self.out_min), ptr(self.samples), stream_ptr()),
              "swarm_train_act_step")

    def launch_td(self):
        check(self.lib.swarm_td_grad(ctypes_ref(self.cfg), ctypes_ref(self.hp), ptr(self.w_nxt), ptr(self.target),
                                     ctypes_ref(self.replay), ptr(self.ctrl), ptr(self.samples), None,
                                     ptr(self.slabs), stream_ptr()), "swarm_td_grad")

    def launch_grad_reduce(self):
        self._grad_dirty = False
        check(self.lib.swarm_grad_reduce(ctypes_ref(self.cfg), ctypes_ref(self.hp), ptr(self.slabs),
                                         ptr(self.grad), stream_ptr()), "swarm_grad_reduce")

    def launch_tick(self, full_out: bool = False):
        """The fused tick's launch (acting + TD blocks); swarm_reduce_advance follows it."""
        self._sync_flags()
        check(self.lib.swarm_train_tick(ctypes_ref(self.cfg), ctypes_ref(self.hp), ctypes_ref(self.learner),
                                        ptr(self.state), ctypes_ref(self.replay), ptr(self.ctrl),
                                        ctypes_ref(self.out if full_out else self.out_min), ptr(self.slabs),
                                        ptr(self.tick_ws), ptr(self.samples), stream_ptr()), "swarm_train_tick")

    def launch_reduce_advance(self):
        """Slab reduce + ctrl advance; with a peer exchange, the gradient all-reduce too."""
        self._grad_dirty = False
        if self.peer is not None:
            self.peer.check_stream()
            check(self.lib.swarm_reduce_advance_peer(ctypes_ref(self.cfg), ctypes_ref(self.hp), ptr(self.slabs),
                                                     ctypes_ref(self.learner), self.capacity, ptr(self.ctrl),
                                                     ctypes_ref(self.peer.struct), stream_ptr()),
                  "swarm_reduce_advance_peer")
            return
        check(self.lib.swarm_reduce_advance(ctypes_ref(self.cfg), ctypes_ref(self.hp), ptr(self.slabs),
                                            ctypes_ref(self.learner), self.capacity, ptr(self.ctrl), stream_ptr()),
              "swarm_reduce_advance")

    def handoff_errors(self) -> int:
        """Hand-off waits of the fused tick that hit their bound (0 in a correct run)."""
        if self.tick_ws is None:
            return 0
        return int(self.tick_ws[:4].view(torch.int32).item())   # the workspace's first word

    def check_handoffs(self):
        """Raise if any fused-tick hand-off wait overran since the workspace was zeroed.  An
        overrun drops the graphs it waited for from that tick's TD batch (their terms are zero,
        the mean stays over S*N nodes), so training never consumes a stale transition; this
        makes the event loud.  One 4-byte device read: call it once per episode."""
        n = self.handoff_errors()
        if n:
            raise RuntimeError(f"fused training tick: {n} hand-off wait(s) overran their bound; the graphs they "
                               "waited for were dropped from their TD batches (use train_tick3 on this device)")

    def train_tick(self, full_out: bool = False):
        """Fused training tick: 2 launches (+ an RCCL all-reduce when world_size > 1), or the
        3-launch tick where no fused-tick kernel exists.  Writes this tick's TD batch
        indices to self.samples."""
        if not self.fused:
            return self.train_tick3(full_out)
        self.launch_tick(full_out)
        self.launch_reduce_advance()
        if self.peer is None:
            self.allreduce_grad()

    def train_tick3(self, full_out: bool = False):
        """3-launch training tick: act (+ this tick's TD batch indices), TD, reduce."""
        self._sync_flags()
        cfg, hp = ctypes_ref(self.cfg), ctypes_ref(self.hp)
        check(self.lib.swarm_train_act_step(cfg, hp, ctypes_ref(self.learner), ptr(self.state),
                                            ctypes_ref(self.replay), ptr(self.ctrl),
                                            ctypes_ref(self.out if full_out else self.out_min), ptr(self.samples),
                                            stream_ptr()), "swarm_train_act_step")
        check(self.lib.swarm_td_grad(cfg, hp, ptr(self.w_nxt), ptr(self.target), ctypes_ref(self.replay),
                                     ptr(self.ctrl), ptr(self.samples), None, ptr(self.slabs), stream_ptr()),
              "swarm_td_grad")
        self.launch_reduce_advance()
        if self.peer is None:
            self.allreduce_grad()

    # ------------------------------------------------------------------ hipGraph
    def capture(self, n_ticks: int, fn=None):
        """Capture n_ticks calls of ``fn`` (default train_tick) into one hipGraph.  With
        world_size > 1 the tick's RCCL all-reduce is captured too; the capture is then
        thread-local so the process group's watchdog thread may keep querying its events."""
        fn = fn or self.train_tick
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream())
        graph = torch.cuda.CUDAGraph()
        mode = "thread_local" if self.world_size > 1 else "global"
        with torch.cuda.stream(s):
            with torch.cuda.graph(graph, stream=s, capture_error_mode=mode):
                for _ in range(n_ticks):
                    fn()
        torch.cuda.current_stream().wait_stream(s)
        return graph

    # ------------------------------------------------------------------ weights
    def state_dict(self) -> dict:
        if self.net == "gcn":
            self.flush()
        return unflatten_params(self.params.detach().cpu(), self.net)

    def load_state_dict(self, sd):
        self.params.copy_(flatten_state_dict(sd, net=self.net).to(self.device))
        self.target.copy_(self.params)


def ctypes_ref(obj):
    import ctypes
    return None if obj is None else ctypes.byref(obj)
