"""PyTorch-CPU fp32 restatement of the reference hot path (TEST INFRASTRUCTURE ONLY).

This module is the *checker* for the HIP path.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it; the product path (``experiments-2025-acsos-marl-for-swarming-behaviors_amd``)
never does and fails loudly when its HIP library is missing.

What it restates (citations relative to the reference checkout):

* VMAS 1.4.0 ``Environment.step`` for the two scenarios (third-party, not vendored;
  ``requirements.txt:3``).  Arithmetic written out in SURVEY.md §8(a) rows a1-a6:
  discrete decode, holonomic force, sphere-sphere collision force
  (``World._sphere_sphere_vectorized_collision`` / ``_get_constraint_forces``),
  drag + Euler integration, then the scenario ``reward`` / ``observation``.
* ``GoToPositionScenario`` (``src/scenarios/go_to_position_scenario.py:52-143``).
* ``ObstacleAvoidanceScenario`` (``src/scenarios/obstacle_avoidance_scenario.py:63-173``).
* ``FlockingScenario`` (``src/scenarios/flocking_scenario.py:9-176``): reset centre and the
  shaped collective reward (``flocking_reward``).  Parity unpinned: the reference holds no
  Flocking trajectories (its ``data/test_stats`` cover GoTo and ObstacleAvoidance only).
* PyG 2.5.3 ``GATConv`` (heads=1, add_self_loops=False, negative_slope=0.2, bias)
  and ``torch_geometric.utils.softmax`` (third-party, ``requirements.txt:2``).
* ``GCN.forward`` (``src/training/train_gcn_dqn.py:59-70``).
* Graph builders: training complete graph (``train_gcn_dqn.py:94-110``) and the
  evaluation kNN graph (``src/simulation/simulator.py:9-26``).
* ``DQNTrainer.train_step_dqn`` (``train_gcn_dqn.py:112-137``): gather, target max,
  MSE, backward, ``clip_grad_norm_(…, 1)``, ``Adam(lr=1e-3)``.
* ε-greedy (``train_gcn_dqn.py:161-169``) with the draws keyed through Philox
  (``oracle/philox.py``) instead of Python ``random``.

Parity pin: ``tests/test_oracle_golden.py`` checks this restatement against the
reference's own recorded evaluation trajectories (``data/test_stats/**``) and
trained weights (``data/models/*.pth``), committed as fixtures under
``tests/golden/`` by ``tests/golden/make_golden.py``.
"""
from __future__ import annotations

import contextlib
import math
from dataclasses import dataclass

import numpy as np
import torch
import torch.nn.functional as F

from . import philox

# ---------------------------------------------------------------------------
# constants
# ---------------------------------------------------------------------------
GOAL = (-0.8, 0.8)              # go_to_position_scenario.py:86, obstacle_avoidance_scenario.py:97
OBSTACLE = (-0.1, 0.1)          # obstacle_avoidance_scenario.py:99
SPHERE_RADIUS = 0.05            # VMAS Sphere() default radius (agents and the obstacle)
COLLISION_FORCE = 100.0         # VMAS World collision_force default
CONTACT_MARGIN = 1e-3           # VMAS World contact_margin default
MIN_DIST = 1e-6                 # VMAS _get_constraint_forces min_dist
DT = 0.1                        # VMAS World dt, substeps=1
DRAG = 0.25                     # VMAS World drag default
GRID_SPACING = 0.15             # desired_distance (go_to_position_scenario.py:17)
FLOCK_SHAPING = 10.0            # flocking_scenario.py:10-11 pos/dist_shaping_factor
FLOCK_DESIRED = 0.15            # flocking_scenario.py:20 desired_distance
FLOCK_CONTACT = 0.005           # flocking_scenario.py:21 min_collision_distance
FLOCK_GOAL_BONUS = 50.0         # flocking_scenario.py:146-147
N_ACTIONS = 9
N_FEATURES = 7
HIDDEN = 32
ACTION_LEVELS = (0.0, -1.0, 1.0)  # discrete level index -> u component

SCENARIO_GOTO = 0
SCENARIO_OA = 1
SCENARIO_FLOCK = 2

PARAM_ORDER = (  # == GCN.parameters() order / state_dict order (PyG registers att, bias, then lin)
    ("conv1.att_src", (1, 1, HIDDEN)),
    ("conv1.att_dst", (1, 1, HIDDEN)),
    ("conv1.bias", (HIDDEN,)),
    ("conv1.lin.weight", (HIDDEN, N_FEATURES)),
    ("lin1.weight", (HIDDEN, HIDDEN)),
    ("lin1.bias", (HIDDEN,)),
    ("lin2.weight", (N_ACTIONS, HIDDEN)),
    ("lin2.bias", (N_ACTIONS,)),
)
N_PARAMS = sum(int(np.prod(s)) for _, s in PARAM_ORDER)  # 1673


def f32(x):
    return torch.as_tensor(x, dtype=torch.float32)


# ---------------------------------------------------------------------------
# parameters
# ---------------------------------------------------------------------------
def flatten_params(sd) -> torch.Tensor:
    return torch.cat([sd[k].reshape(-1).to(torch.float32) for k, _ in PARAM_ORDER])


def unflatten_params(flat) -> dict:
    flat = torch.as_tensor(flat, dtype=torch.float32)
    out, o = {}, 0
    for k, shape in PARAM_ORDER:
        n = int(np.prod(shape))
        out[k] = flat[o:o + n].reshape(shape).clone()
        o += n
    return out


# ---------------------------------------------------------------------------
# env step  (VMAS World.step + scenario reward/observation)
# ---------------------------------------------------------------------------
def decode_actions(actions: torch.Tensor) -> torch.Tensor:
    """a in 0..8 -> u = (L[a // 3], L[a % 3]), L = [0, -1, +1]."""
    lv = torch.tensor(ACTION_LEVELS, dtype=torch.float32)
    a = actions.to(torch.long)
    return torch.stack([lv[a // 3], lv[a % 3]], dim=-1)


def vector_norm2(d: torch.Tensor) -> torch.Tensor:
    """torch.linalg.vector_norm over the last dim of size 2 (what VMAS/the scenarios call)."""
    return torch.linalg.vector_norm(d, dim=-1)


def pair_force(pos_a: torch.Tensor, pos_b: torch.Tensor, dist_min: float = 2 * SPHERE_RADIUS):
    """VMAS _get_constraint_forces (attractive=False): force on a; force on b is its negation."""
    delta = pos_a - pos_b
    dist = vector_norm2(delta)
    k = CONTACT_MARGIN
    dmin = torch.full_like(dist, SPHERE_RADIUS) + torch.full_like(dist, SPHERE_RADIUS)
    pen = torch.logaddexp(torch.tensor(0.0), (dmin - dist) * 1 / k) * k
    force = COLLISION_FORCE * delta / torch.where(dist > 0, dist, torch.tensor(1e-8)).unsqueeze(-1) * pen.unsqueeze(-1)
    force = torch.where((dist < MIN_DIST).unsqueeze(-1), torch.tensor(0.0), force)
    force = torch.where((dist > dmin).unsqueeze(-1), torch.tensor(0.0), force)
    return force


def env_step(pos: torch.Tensor, vel: torch.Tensor, actions: torch.Tensor, scenario: int,
             prev_spread: torch.Tensor | None = None):
    """One VMAS step for [B, N] agents.  Returns dict of new state, rewards and metrics.

    Flocking keeps per-agent state (``previous_distance_to_agents``): ``prev_spread`` [B, N]
    is its value before the step (``flocking_reset_spread`` right after a reset; None = the
    shaped spread of ``pos``, which is what every later step stores), and the returned
    dict's ``spread`` is the value after it.

    Force summation order follows VMAS: force = 0 + u, then the obstacle pair
    (landmarks precede agents in ``world.entities``), then agent pairs (a<b) in
    lexicographic order, i.e. ascending partner index for every agent.
    """
    pos = pos.to(torch.float32)
    vel = vel.to(torch.float32)
    B, N, _ = pos.shape
    force = torch.zeros(B, N, 2) + decode_actions(actions)
    obst = f32(OBSTACLE)
    if scenario == SCENARIO_OA:
        # pair (obstacle, agent_j): obstacle is entity_a -> agent receives -force_a
        fa = pair_force(obst.expand(B, N, 2), pos)
        force = force + (-fa)
    for v in range(N):
        acc = force[:, v]
        for u in range(N):
            if u == v:
                continue
            if u < v:   # pair (u, v): v is entity_b -> receives -force(p_u - p_v)
                acc = acc + (-pair_force(pos[:, u], pos[:, v]))
            else:       # pair (v, u): v is entity_a
                acc = acc + pair_force(pos[:, v], pos[:, u])
        force[:, v] = acc
    vel_new = vel * (1 - DRAG)
    accel = force / 1.0
    vel_new = vel_new + accel * DT
    pos_new = pos + vel_new * DT
    goal = f32(GOAL)
    dist_goal = vector_norm2(pos_new - goal)                    # [B, N]
    if scenario == SCENARIO_FLOCK:
        rew, hits, spread = flocking_reward(pos, pos_new, prev_spread)
        d_obs = torch.zeros(B, N)
    elif scenario == SCENARIO_GOTO:
        r = torch.zeros(B)
        acc = None
        for j in range(N):                                      # go_to_position_scenario.py:108-115
            acc = -dist_goal[:, j] if acc is None else acc + (-dist_goal[:, j])
        rew = acc.unsqueeze(1).expand(B, N).clone()
        d_obs = torch.zeros(B, N)
        hits = torch.zeros(B)
    else:
        d_obs = (vector_norm2(pos_new - obst) - SPHERE_RADIUS) - SPHERE_RADIUS   # World.get_distance
        obst_rew = torch.where(d_obs <= 1, -(1 - d_obs), torch.tensor(0.0))      # obstacle_avoidance_scenario.py:146-152
        rew = -dist_goal + 2.5 * obst_rew
        hits = (d_obs <= 0.2).sum(dim=1).to(torch.float32)                       # obstacle_avoidance_scenario.py:170-173
    avg_dist = torch.mean(dist_goal, dim=1)
    out = dict(pos=pos_new, vel=vel_new, force=force, rew=rew, dist_goal=dist_goal,
               avg_dist=avg_dist, hits=hits, d_obs=d_obs)
    if scenario == SCENARIO_FLOCK:
        out["spread"] = spread
    return out


def _flock_agent_spread(pos: torch.Tensor, i: int) -> torch.Tensor:
    """flocking_scenario.py:151-162 (and :110-122): mean over the other agents of
    (|p_i - p_j| - desired)^2, times dist_shaping_factor."""
    N = pos.shape[1]
    d = torch.stack([vector_norm2(pos[:, i] - pos[:, j]) for j in range(N) if j != i], dim=1)
    return (d - FLOCK_DESIRED).pow(2).mean(-1) * FLOCK_SHAPING


def flocking_reset_spread(pos: torch.Tensor) -> torch.Tensor:
    """``previous_distance_to_agents`` as ``reset_world_at`` leaves it (flocking_scenario.py:93-122).

    The reset loop places agent i and computes its spread in the same iteration, so agents
    j < i are already at their new positions while agents j > i are still where VMAS's
    ``env_reset_world_at`` put them: ``World.reset`` zeroes every entity state before the
    scenario's ``reset_world_at`` runs (VMAS 1.4.0), i.e. the origin.  [B, N] fp32."""
    B, N, _ = pos.shape
    out = torch.zeros(B, N)
    zero = torch.zeros(B, 2)
    for i in range(N):
        d = torch.stack([vector_norm2(pos[:, i] - (pos[:, j] if j < i else zero)) for j in range(N) if j != i], dim=1)
        out[:, i] = (d - FLOCK_DESIRED).pow(2).mean(-1) * FLOCK_SHAPING
    return out


def flocking_reward(pos: torch.Tensor, pos_new: torch.Tensor, prev_spread: torch.Tensor | None = None):
    """FlockingScenario.reward (flocking_scenario.py:124-176) for [B, N] agents.

    The scenario keeps ``previous_distance_to_goal`` / ``previous_distance_to_agents`` per
    agent.  The goal term's stored value is always the shaped distance of the pre-step
    position (set at reset :102-107 from the agent's new position, then by every reward call
    :140-142), so it is recomputed from ``pos``.  The spread's stored value is the previous
    reward call's (:163-164) except on the first step after a reset, where it is
    ``flocking_reset_spread``'s mixed old/new value: the caller passes it as ``prev_spread``
    (None = recompute from ``pos``, the later steps' value).
    ``if agent.on_goal`` only works at B=1 in the reference; this is its batched form.
    Returns (collective reward broadcast to [B, N], contact count per env, spread after [B, N])."""
    B, N, _ = pos.shape
    goal = f32(GOAL)
    total, contacts = None, torch.zeros(B)
    spread = torch.zeros(B, N)
    for i in range(N):
        d_now = vector_norm2(pos_new[:, i] - goal)
        pos_rew = vector_norm2(pos[:, i] - goal) * FLOCK_SHAPING - d_now * FLOCK_SHAPING
        r_goal = torch.where(d_now < SPHERE_RADIUS, pos_rew + FLOCK_GOAL_BONUS, pos_rew)
        cnt = torch.zeros(B)
        for j in range(N):
            if j != i:   # World.get_distance(agent, other) <= min_collision_distance
                gd = (vector_norm2(pos_new[:, i] - pos_new[:, j]) - SPHERE_RADIUS) - SPHERE_RADIUS
                cnt = cnt + (gd <= FLOCK_CONTACT).to(torch.float32)
        before = _flock_agent_spread(pos, i) if prev_spread is None else prev_spread[:, i]
        spread[:, i] = _flock_agent_spread(pos_new, i)
        dist_rew = before - spread[:, i]
        term = (r_goal + (-cnt)) + dist_rew
        total = term if total is None else total + term
        contacts = contacts + cnt
    return total.unsqueeze(1).expand(B, N).clone(), contacts, spread


def flocking_reward_scale(pos: torch.Tensor, pos_new: torch.Tensor,
                          prev_spread: torch.Tensor | None = None) -> torch.Tensor:
    """[B] sum of the magnitudes the flocking reward is a difference of (shaped goal distances
    and spreads, before and after the step).  The reward cancels most of it, so its fp32
    rounding is bounded relative to this scale, not to the reward itself."""
    goal = f32(GOAL)
    N = pos.shape[1]
    s = torch.zeros(pos.shape[0], dtype=torch.float64)
    for i in range(N):
        for p in (pos, pos_new):
            s += (vector_norm2(p[:, i] - goal) * FLOCK_SHAPING).double() + _flock_agent_spread(p, i).double()
        if prev_spread is not None:
            s += prev_spread[:, i].double()
    return s


# ---------------------------------------------------------------------------
# reset  (generate_grid + reset_world_at)
# ---------------------------------------------------------------------------
def grid_offsets(n_agents: int):
    """go_to_position_scenario.py:52-80: row-major grid, cols = ceil(sqrt(N))."""
    cols = math.ceil(math.sqrt(n_agents))
    rows = math.ceil(n_agents / cols)
    offs = []
    for i in range(rows):
        for j in range(cols):
            offs.append(((j - (cols - 1) / 2) * GRID_SPACING, (i - (rows - 1) / 2) * GRID_SPACING))
            if len(offs) >= n_agents:
                break
        if len(offs) >= n_agents:
            break
    return np.asarray(offs, dtype=np.float64)


def grid_positions(centres: torch.Tensor, n_agents: int) -> torch.Tensor:
    """centres [B,2] fp32 -> pos [B,N,2]; x = c + fp32(offset) (tensor + python float)."""
    offs = torch.tensor(grid_offsets(n_agents), dtype=torch.float64).to(torch.float32)
    return centres.to(torch.float32)[:, None, :] + offs[None, :, :]


def reset_centres(scenario: int, n_envs: int, seed: int, episode: int, shared: bool, random_oa: bool = True,
                  env_offset: int = 0):
    """Reset centres with Philox + Box-Muller in float64 (the HIP reset kernel uses
    fp32 libm calls, so reset positions are compared with a tolerance).  Draws are
    keyed by the GLOBAL env index env_offset + e (rank sharding)."""
    k0, k1 = philox.seed_key(seed)
    envs = (np.zeros(n_envs, dtype=np.uint32) if shared
            else np.arange(n_envs, dtype=np.uint32) + np.uint32(env_offset))
    w = philox.philox4x32(np.uint32(episode), envs, philox.STREAM_RESET, 0, k0, k1)
    u1 = ((w[0] >> np.uint32(8)).astype(np.float64) + 1.0) * 2.0 ** -24
    u2 = (w[1] >> np.uint32(8)).astype(np.float64) * 2.0 ** -24
    rr = np.sqrt(-2.0 * np.log(u1))
    z0, z1 = rr * np.cos(2 * np.pi * u2), rr * np.sin(2 * np.pi * u2)
    if scenario == SCENARIO_FLOCK:  # flocking_scenario.py:86-91: [-1, 1] + N((-0.6,0.6), 0.4)
        cx = np.float32(-1.0) + (np.float32(-0.6) + np.float32(0.4) * z0.astype(np.float32))
        cy = np.float32(1.0) + (np.float32(0.6) + np.float32(0.4) * z1.astype(np.float32))
    elif scenario == SCENARIO_GOTO:   # (1.5,-1.5) + N((-0.6,0.6), 0.4)
        cx = np.float32(1.5) + (np.float32(-0.6) + np.float32(0.4) * z0.astype(np.float32))
        cy = np.float32(-1.5) + (np.float32(0.6) + np.float32(0.4) * z1.astype(np.float32))
    else:                           # (0.6,-0.6) + (random ? N(0,0.1) : 0)
        s = np.float32(0.1) if random_oa else np.float32(0.0)
        cx = np.float32(0.6) + s * z0.astype(np.float32)
        cy = np.float32(-0.6) + s * z1.astype(np.float32)
    return torch.tensor(np.stack([cx, cy], axis=1).astype(np.float32))


def reset_from_first_step(P0, P1, scenario: int, window: int = 64):
    """The reset formation an evaluation episode started from, recovered from its first two
    recorded positions (test infrastructure: the reference re-seeds torch and draws its reset
    centre from a stream this build cannot reproduce, SURVEY §8(c), but its Simulator records
    every tick's positions after the step, simulator.py:59-84).

    At reset the agents stand on the generate_grid formation around a centre c with v = 0
    (go_to_position_scenario.py:52-106, obstacle_avoidance_scenario.py:63-133); the grid spacing
    (0.15) exceeds the contact distance (0.1) and the obstacle is far, so the first step has no
    collision force: v1 = dt u0 and P0 = p0 + dt v1.  The centre is unknown, so P0 alone cannot
    tell a common u0 from a shifted centre; the second step can: (P1 - P0) / dt - dt f(P0) =
    0.75 dt u0 + dt u1 (VMAS drag 0.25, f the collision force at P0), and 0.075 a + 0.1 b takes a
    different value for each of the nine level pairs (a, b).  With u0 known, p0 is the fp32 value
    next to P0 - dt v1 whose first step reproduces P0 exactly (checked with env_step, as is the
    grid: P0 - dt v1 - offset agrees on one centre).  P0, P1 [N, 2] fp32.
    Returns (p0 [N, 2] fp32, u0 as actions [N] long)."""
    P0 = np.asarray(P0, dtype=np.float32)
    P1 = np.asarray(P1, dtype=np.float32)
    N = P0.shape[0]
    f1 = env_step(torch.tensor(P0)[None], torch.zeros(1, N, 2), torch.zeros(1, N, dtype=torch.long),
                  scenario)["force"][0].double().numpy()                          # action 0: u = 0, force = f(P0)
    x = (P1.astype(np.float64) - P0.astype(np.float64)) / DT - DT * f1           # 0.075 u0 + 0.1 u1 per axis
    lv = np.array(ACTION_LEVELS)
    combos = np.array([[0.75 * DT * a0 + DT * a1 for a1 in lv] for a0 in lv])     # [u0 level][u1 level]
    lidx = np.zeros((N, 2), dtype=np.int64)
    for i in range(N):
        for k in range(2):
            err = np.abs(combos - x[i, k])
            j0, j1 = np.unravel_index(int(np.argmin(err)), err.shape)
            if err[j0, j1] > 1e-3 or np.sort(err.ravel())[1] < 1e-2:
                raise ValueError("the first two recorded steps do not determine the first action")
            lidx[i, k] = j0
    acts = (3 * lidx[:, 0] + lidx[:, 1]).tolist()
    offs = grid_offsets(N)
    centres = P0.astype(np.float64) - 0.01 * lv[lidx] - offs
    if np.abs(centres - centres[0]).max() > 1e-4:
        raise ValueError("the first recorded positions are not one step from a grid formation")
    a = torch.tensor(acts, dtype=torch.long)
    u = decode_actions(a).numpy()
    step = (u * np.float32(DT)).astype(np.float32) * np.float32(DT)   # vel_new * dt with vel_new = 0 * 0.75 + u * dt
    p0 = np.empty_like(P0)
    for i in range(N):
        for k in range(2):
            x = np.float32(P0[i, k] - step[i, k])
            for _ in range(window):   # walk to an fp32 value whose step lands exactly on P0
                y = np.float32(x + step[i, k])
                if y == P0[i, k]:
                    break
                x = np.nextafter(x, np.float32(np.inf if y < P0[i, k] else -np.inf), dtype=np.float32)
            p0[i, k] = x
    p0t = torch.tensor(p0)
    got = env_step(p0t[None], torch.zeros(1, N, 2), a[None], scenario)["pos"][0]
    if not torch.equal(got, torch.tensor(P0)):
        raise ValueError("no fp32 reset formation reproduces the first recorded step")
    return p0t, a


def episode_result(rew, avg_dist, hits):
    """One result.csv row of an evaluation episode as the reference's Simulator forms it
    (simulator.py:59-109): Reward = (sum over ticks of the python sum of the agents' fp32
    rewards) / max_steps, accumulated in fp32 in that order; Collisions = the summed per-tick
    obstacle hits; Distance (end) / (beginning) = average_distance_to_goal() after the last /
    the first step.  rew [T, N] fp32 per agent and tick, avg_dist [T], hits [T].
    Returns (reward, collisions, distance end, distance beginning) as Python floats."""
    rew = torch.as_tensor(rew, dtype=torch.float32)
    T, N = rew.shape
    total = torch.zeros((), dtype=torch.float32)
    for t in range(T):
        s = torch.zeros((), dtype=torch.float32)   # sum(rewards.values()) starts from int 0
        for i in range(N):
            s = s + rew[t, i]
        total = total + s
    avg_dist = torch.as_tensor(avg_dist, dtype=torch.float32)
    return (float(total / T), float(torch.as_tensor(hits, dtype=torch.float64).sum()), float(avg_dist[-1]),
            float(avg_dist[0]))


# ---------------------------------------------------------------------------
# observations / node features
# ---------------------------------------------------------------------------
def node_features(pos: torch.Tensor, vel: torch.Tensor) -> torch.Tensor:
    """[B,N,7] = [pos, vel, goal, float(agent id)] (train_gcn_dqn.py:94-99)."""
    B, N, _ = pos.shape
    goal = f32(GOAL).expand(B, N, 2)
    ids = torch.arange(N, dtype=torch.float32).view(1, N, 1).expand(B, N, 1)
    return torch.cat([pos, vel, goal, ids], dim=-1)


# ---------------------------------------------------------------------------
# graph builders
# ---------------------------------------------------------------------------
def complete_edge_index(n: int) -> torch.Tensor:
    """train_gcn_dqn.py:101-108: (i,j),(j,i) for i<j, then [0,0]."""
    e = []
    for i in range(n):
        for j in range(i + 1, n):
            e.append([i, j])
            e.append([j, i])
    e.append([0, 0])
    return torch.tensor(e, dtype=torch.long).t().contiguous()


def knn_edge_index(pos: torch.Tensor, k: int) -> torch.Tensor:
    """simulator.py:15-24 for one env: pos [N,2] fp32."""
    n = pos.shape[0]
    e = []
    for i in range(n):
        d = torch.linalg.norm(pos[:, :2] - pos[i, :2], dim=1)
        _, nearest = torch.topk(d, k, largest=False)
        for a in nearest:
            e.append([i, a.item()])
            e.append([a.item(), i])
    e.append([0, 0])
    return torch.tensor(e, dtype=torch.long).t().contiguous()


def knn_sets(pos: torch.Tensor, k: int) -> torch.Tensor:
    """[B,N,2] -> bool [B, N(i), N(j)]: j in kNN(i), via the reference's own topk call."""
    B, N, _ = pos.shape
    out = torch.zeros(B, N, N, dtype=torch.bool)
    for b in range(B):
        for i in range(N):
            d = torch.linalg.norm(pos[b, :, :2] - pos[b, i, :2], dim=1)
            _, idx = torch.topk(d, k, largest=False)
            out[b, i, idx] = True
    return out


def radius_sets(pos: torch.Tensor, radius: float) -> torch.Tensor:
    """[B,N,2] -> bool [B, N(i), N(j)]: j != i with |p_j - p_i| <= radius.  The radius-neighbour
    graph of the north_star (not in the reference, SURVEY §8(f) row 3: parity unpinned); the
    distance is the kNN build's own expression (simulator.py:18) so the sets are bit-exact."""
    B, N, _ = pos.shape
    out = torch.zeros(B, N, N, dtype=torch.bool)
    r = torch.tensor(radius, dtype=torch.float32)
    for b in range(B):
        for i in range(N):
            d = torch.linalg.norm(pos[b, :, :2] - pos[b, i, :2], dim=1)
            out[b, i] = d <= r
            out[b, i, i] = False
    return out


def radius_edge_index(pos: torch.Tensor, radius: float) -> torch.Tensor:
    """Edge-list form for one env (pos [N,2]): (i, j) for j in R(i), then (0, 0)."""
    s = radius_sets(pos[None], radius)[0]
    e = [[i, j] for i in range(pos.shape[0]) for j in range(pos.shape[0]) if bool(s[i, j])]
    e.append([0, 0])
    return torch.tensor(e, dtype=torch.long).t().contiguous()


def multiplicity_radius(sets: torch.Tensor) -> torch.Tensor:
    """m(u->v) = [v in R(u)] + [u=v=0]; R is symmetric, so every ordered pair appears once."""
    m = sets.to(torch.float32).clone()
    m[:, 0, 0] += 1.0
    return m


def multiplicity_complete(B: int, N: int) -> torch.Tensor:
    """m[b,u,v] = #edges u->v of the training graph."""
    m = torch.ones(B, N, N) - torch.eye(N).expand(B, N, N)
    m[:, 0, 0] = 1.0
    return m


def multiplicity_knn(sets: torch.Tensor) -> torch.Tensor:
    """m(u->v) = [v in S_u] + [u in S_v] + [u=v=0]  (edges (i,j),(j,i) per j in S_i)."""
    s = sets.to(torch.float32)
    m = s + s.transpose(1, 2)
    m[:, 0, 0] += 1.0
    return m


def edge_index_from_multiplicity(m: torch.Tensor) -> torch.Tensor:
    """Batched multiplicity [B,N,N] -> PyG-style concatenated edge_index (duplicates expanded)."""
    B, N, _ = m.shape
    src, dst = [], []
    for b in range(B):
        for u in range(N):
            for v in range(N):
                for _ in range(int(m[b, u, v].item())):
                    src.append(b * N + u)
                    dst.append(b * N + v)
    return torch.tensor([src, dst], dtype=torch.long)


# ---------------------------------------------------------------------------
# GAT / GCN forward
# ---------------------------------------------------------------------------
def gat_conv_edges(x, edge_index, W, att_src, att_dst, bias):
    """PyG 2.5.3 GATConv(heads=1, add_self_loops=False) on an explicit edge list.

    alpha_e = softmax_dst(leaky_relu(a_src[src] + a_dst[dst], 0.2)) with the
    max taken over detached scores and a +1e-16 denominator; out = scatter_add
    over dst of alpha * h[src]; + bias.
    """
    M = x.shape[0]
    h = F.linear(x, W)                                           # lin (no bias)
    a_s = (h * att_src.reshape(1, -1)).sum(-1)
    a_d = (h * att_dst.reshape(1, -1)).sum(-1)
    src, dst = edge_index[0], edge_index[1]
    e = a_s[src] + a_d[dst]
    e = F.leaky_relu(e, 0.2)
    emax = torch.zeros(M, dtype=e.dtype).scatter_reduce(0, dst, e.detach(), reduce="amax", include_self=False)
    ex = (e - emax[dst]).exp()
    den = torch.zeros(M, dtype=e.dtype).scatter_add(0, dst, ex) + 1e-16
    alpha = ex / den[dst]
    msg = alpha.unsqueeze(-1) * h[src]
    out = torch.zeros(M, h.shape[1], dtype=h.dtype).scatter_add(0, dst.unsqueeze(-1).expand_as(msg), msg)
    return out + bias


def q_forward_edges(params: dict, x: torch.Tensor, edge_index: torch.Tensor) -> torch.Tensor:
    """GCN.forward (train_gcn_dqn.py:59-70) on an edge list."""
    g = gat_conv_edges(x, edge_index, params["conv1.lin.weight"], params["conv1.att_src"],
                       params["conv1.att_dst"], params["conv1.bias"])
    t = torch.tanh(g)
    z = torch.relu(F.linear(t, params["lin1.weight"], params["lin1.bias"]))
    return F.linear(z, params["lin2.weight"], params["lin2.bias"])


def q_forward_dense(params: dict, x: torch.Tensor, mult: torch.Tensor, return_all: bool = False):
    """Vectorised [B,N] restatement with a dense edge-multiplicity matrix mult[b,u,v].

    Equals q_forward_edges on edge_index_from_multiplicity(mult) up to fp32
    summation order (tests/test_oracle_internal.py checks it).
    """
    W = params["conv1.lin.weight"]
    h = F.linear(x, W)                                           # [B,N,H]
    a_s = (h * params["conv1.att_src"].reshape(1, 1, -1)).sum(-1)
    a_d = (h * params["conv1.att_dst"].reshape(1, 1, -1)).sum(-1)
    e = F.leaky_relu(a_s[:, :, None] + a_d[:, None, :], 0.2)     # [B,u,v]
    present = mult > 0
    neg = torch.tensor(float("-inf"))
    emax = torch.where(present, e.detach(), neg).amax(dim=1)     # [B,v]
    emax = torch.where(torch.isinf(emax), torch.zeros_like(emax), emax)
    ex = torch.where(present, (e - emax[:, None, :]).exp(), torch.zeros_like(e))
    den = (mult * ex).sum(dim=1) + 1e-16                         # [B,v]
    alpha = ex / den[:, None, :]
    out = torch.einsum("buv,buh->bvh", mult * alpha, h) + params["conv1.bias"]
    t = torch.tanh(out)
    z = torch.relu(F.linear(t, params["lin1.weight"], params["lin1.bias"]))
    q = F.linear(z, params["lin2.weight"], params["lin2.bias"])
    if return_all:
        return dict(h=h, a_s=a_s, a_d=a_d, alpha=alpha, out=out, t=t, z=z, q=q)
    return q


def gat_conv_dense(x: torch.Tensor, mult: torch.Tensor, W, att_src, att_dst, bias) -> torch.Tensor:
    """One GATConv of q_forward_dense for [B,N] graphs (any width)."""
    h = F.linear(x, W)
    a_s = (h * att_src.reshape(1, 1, -1)).sum(-1)
    a_d = (h * att_dst.reshape(1, 1, -1)).sum(-1)
    e = F.leaky_relu(a_s[:, :, None] + a_d[:, None, :], 0.2)
    present = mult > 0
    emax = torch.where(present, e.detach(), torch.tensor(float("-inf"))).amax(dim=1)
    emax = torch.where(torch.isinf(emax), torch.zeros_like(emax), emax)
    ex = torch.where(present, (e - emax[:, None, :]).exp(), torch.zeros_like(e))
    den = (mult * ex).sum(dim=1) + 1e-16
    return torch.einsum("buv,buh->bvh", mult * (ex / den[:, None, :]), h) + bias


GAT3_PARAM_ORDER = tuple(
    (f"conv{i}.{n}", s) for i, k in ((1, 7), (2, 8), (3, 8))
    for n, s in (("att_src", (1, 1, 8)), ("att_dst", (1, 1, 8)), ("bias", (8,)), ("lin.weight", (8, k))))
GAT3_PARAM_ORDER += (("lin1.weight", (8, 8)), ("lin1.bias", (8,)), ("lin2.weight", (9, 8)), ("lin2.bias", (9,)))
GAT3_N_PARAMS = sum(int(np.prod(s)) for _, s in GAT3_PARAM_ORDER)   # 409


def gat3_unflatten(flat) -> dict:
    flat = torch.as_tensor(flat, dtype=torch.float32)
    out, o = {}, 0
    for k, shape in GAT3_PARAM_ORDER:
        n = int(np.prod(shape))
        out[k] = flat[o:o + n].reshape(shape).clone()
        o += n
    return out


def gat3_q_forward_edges(params: dict, x: torch.Tensor, edge_index: torch.Tensor) -> torch.Tensor:
    """The Flocking checkpoints' network (data/models/experiment_Flocking-seed_*.pth): GCN.forward
    with its commented layers (train_gcn_dqn.py:54-55, 62-70): conv1 -> tanh -> conv2 -> relu
    -> conv3 -> relu -> lin1 -> relu -> lin2, hidden 8.  Parity unpinned (no recorded Flocking
    outputs); the checkpoints' shapes are the architecture's only pin."""
    def conv(i, z):
        return gat_conv_edges(z, edge_index, params[f"conv{i}.lin.weight"], params[f"conv{i}.att_src"],
                              params[f"conv{i}.att_dst"], params[f"conv{i}.bias"])
    z = torch.tanh(conv(1, x))
    z = torch.relu(conv(2, z))
    z = torch.relu(conv(3, z))
    z = torch.relu(F.linear(z, params["lin1.weight"], params["lin1.bias"]))
    return F.linear(z, params["lin2.weight"], params["lin2.bias"])


def gat3_q_forward_dense(params: dict, x: torch.Tensor, mult: torch.Tensor) -> torch.Tensor:
    """gat3_q_forward_edges for [B,N] graphs given by a dense multiplicity."""
    def conv(i, z):
        return gat_conv_dense(z, mult, params[f"conv{i}.lin.weight"], params[f"conv{i}.att_src"],
                              params[f"conv{i}.att_dst"], params[f"conv{i}.bias"])
    z = torch.tanh(conv(1, x))
    z = torch.relu(conv(2, z))
    z = torch.relu(conv(3, z))
    z = torch.relu(F.linear(z, params["lin1.weight"], params["lin1.bias"]))
    return F.linear(z, params["lin2.weight"], params["lin2.bias"])


def gcn_conv_dense(params: dict, x: torch.Tensor, mult: torch.Tensor):
    """a13 (PARITY UNPINNED, not in the reference): PyG 2.5.3 GCNConv defaults on the
    same multigraph: add_remaining_self_loops (self loops collapse to one weight-1
    loop per node), deg counted on targets with duplicates, sym deg^-1/2 norm."""
    W = params["conv1.lin.weight"]
    h = F.linear(x, W)
    B, N, _ = mult.shape
    eye = torch.eye(N).expand(B, N, N)
    # add_remaining_self_loops: existing (duplicate) self loops are dropped and one
    # weight-1 loop per node is appended
    m = mult * (1 - eye) + eye
    deg = m.sum(dim=1)                                           # in-degree per target v
    dis = deg.pow(-0.5)
    dis = torch.where(torch.isinf(dis), torch.zeros_like(dis), dis)
    norm = dis[:, :, None] * m * dis[:, None, :]
    out = torch.einsum("buv,buh->bvh", norm, h) + params["conv1.bias"]
    t = torch.tanh(out)
    z = torch.relu(F.linear(t, params["lin1.weight"], params["lin1.bias"]))
    return F.linear(z, params["lin2.weight"], params["lin2.bias"])


def gcn_conv_edges(params: dict, x: torch.Tensor, edge_index: torch.Tensor, n_nodes: int) -> torch.Tensor:
    """a13 in PyG's own edge-list arithmetic (GCNConv 2.5.3, parity unpinned): gcn_norm with
    add_remaining_self_loops (every self loop dropped, one weight-1 loop per node appended),
    deg = scatter_add of the edge weights on the target, norm = deg^-1/2[src] * w * deg^-1/2[dst],
    then out = scatter_add over edges of norm * h[src] + bias, tanh, lin1, relu, lin2.  The same
    math as gcn_conv_dense, each term formed and summed in a different order: a second fp32
    evaluation of the gradient (tests/test_gpu_parity_large.py).  x [M, 7], edge_index [2, E]."""
    W = params["conv1.lin.weight"]
    h = F.linear(x, W)
    src, dst = edge_index[0], edge_index[1]
    keep = src != dst
    loops = torch.arange(n_nodes)
    src = torch.cat([src[keep], loops])
    dst = torch.cat([dst[keep], loops])
    w = torch.ones(src.shape[0], dtype=h.dtype)
    deg = torch.zeros(n_nodes, dtype=h.dtype).scatter_add_(0, dst, w)
    dis = deg.pow(-0.5)
    dis = torch.where(torch.isinf(dis), torch.zeros_like(dis), dis)
    norm = dis[src] * w * dis[dst]
    out = torch.zeros(n_nodes, h.shape[1], dtype=h.dtype).index_add_(0, dst, norm[:, None] * h[src])
    out = out + params["conv1.bias"]
    t = torch.tanh(out)
    z = torch.relu(F.linear(t, params["lin1.weight"], params["lin1.bias"]))
    return F.linear(z, params["lin2.weight"], params["lin2.bias"])


def argmax_first(q: torch.Tensor) -> torch.Tensor:
    """torch.argmax semantics (first maximal index)."""
    return torch.argmax(q, dim=-1)


# ---------------------------------------------------------------------------
# ε-greedy with Philox draws
# ---------------------------------------------------------------------------
def egreedy(q: torch.Tensor, eps: float, seed: int, tick: int, env_offset: int = 0):
    """One coin per env per tick; if coin < eps every agent draws uniform 0..8.

    q: [B,N,9].  The reference draws one coin per tick for all agents of its
    single env (train_gcn_dqn.py:164-167); the build keys it per env.
    """
    B, N, _ = q.shape
    k0, k1 = philox.seed_key(seed)
    envs = np.arange(B, dtype=np.uint32) + np.uint32(env_offset)
    w = philox.philox4x32(np.uint32(tick), envs, philox.STREAM_COIN, 0, k0, k1)
    coin = torch.tensor(philox.u01(w[0]))
    explore = coin < torch.tensor(np.float32(eps))
    rnd = torch.zeros(B, N, dtype=torch.long)
    for g in range((N + 3) // 4):
        wr = philox.philox4x32(np.uint32(tick), envs, philox.STREAM_RAND_ACTION, np.uint32(g), k0, k1)
        for j in range(4):
            i = 4 * g + j
            if i < N:
                rnd[:, i] = torch.tensor(philox.uniform_int(wr[j], N_ACTIONS))
    greedy = argmax_first(q)
    act = torch.where(explore[:, None], rnd, greedy)
    return act, explore, greedy


# ---------------------------------------------------------------------------
# fused acting tick (graph -> GAT -> eps-greedy -> env step)
# ---------------------------------------------------------------------------
GRAPH_COMPLETE = 0
GRAPH_KNN = 1
GRAPH_RADIUS = 3     # include/swarm_hip.h (2 = caller-supplied dense multiplicity)


@dataclass
class TickOut:
    q: torch.Tensor
    actions: torch.Tensor
    explore: torch.Tensor
    greedy: torch.Tensor
    step: dict
    mult: torch.Tensor


def graph_multiplicity(pos, graph: int, k: int = 0, radius: float = 0.0) -> torch.Tensor:
    B, N, _ = pos.shape
    if graph == GRAPH_COMPLETE:
        return multiplicity_complete(B, N)
    if graph == GRAPH_RADIUS:
        return multiplicity_radius(radius_sets(pos, radius))
    return multiplicity_knn(knn_sets(pos, k))


def act_tick(params: dict, pos, vel, scenario: int, graph: int, k: int, eps: float,
             seed: int, tick: int, conv: str = "gat", env_offset: int = 0, radius: float = 0.0,
             prev_spread=None) -> TickOut:
    B, N, _ = pos.shape
    x = node_features(pos, vel)
    mult = graph_multiplicity(pos, graph, k, radius)
    if "conv2.lin.weight" in params:   # the three-layer GAT (Flocking checkpoints)
        q = gat3_q_forward_dense(params, x, mult)
    elif conv == "gat":
        q = q_forward_dense(params, x, mult)
    else:
        q = gcn_conv_dense(params, x, mult)
    act, explore, greedy = egreedy(q, eps, seed, tick, env_offset)
    step = env_step(pos, vel, act, scenario, prev_spread)
    return TickOut(q=q, actions=act, explore=explore, greedy=greedy, step=step, mult=mult)


# ---------------------------------------------------------------------------
# replay sampling (Feistel permutation; csrc swarm_sample_index)
# ---------------------------------------------------------------------------
def _mix32(x: int) -> int:
    """lowbias32 integer mixer (csrc swarm_common.h mix32)."""
    x &= 0xFFFFFFFF
    x ^= x >> 16
    x = (x * 0x7FEB352D) & 0xFFFFFFFF
    x ^= x >> 15
    x = (x * 0x846CA68B) & 0xFFFFFFFF
    x ^= x >> 16
    return x


def sample_index(i: int, n: int, seed: int, rnd: int) -> int:
    """i-th element of a keyed pseudo-random permutation of [0, n): 4-round alternating
    Feistel on a 2^bits domain, round function mix32(half ^ round_key), round keys =
    one Philox block keyed by (seed, rnd); cycle walking back into [0, n)."""
    k0, k1 = philox.seed_key(seed)
    rk = [int(w) for w in philox.philox4x32(np.uint32(rnd), 0, philox.STREAM_SAMPLE, 0, k0, k1)]
    bits = 2
    while bits < 32 and (1 << bits) < n:
        bits += 1
    lo_bits = bits // 2
    hi_bits = bits - lo_bits
    lo_mask, hi_mask = (1 << lo_bits) - 1, (1 << hi_bits) - 1
    x = i
    while True:
        L, R = x >> lo_bits, x & lo_mask
        R ^= _mix32(L ^ rk[0]) & lo_mask
        L ^= _mix32(R ^ rk[1]) & hi_mask
        R ^= _mix32(L ^ rk[2]) & lo_mask
        L ^= _mix32(R ^ rk[3]) & hi_mask
        x = (L << lo_bits) | R
        if x < n:
            return x


# ---------------------------------------------------------------------------
# TD step (train_gcn_dqn.py:112-137) with torch autograd / clip / Adam
# ---------------------------------------------------------------------------
def complete_batch_edge_index(S: int, N: int) -> torch.Tensor:
    """Batch.from_data_list of S complete graphs (edge offsets by node count)."""
    base = complete_edge_index(N)
    return torch.cat([base + s * N for s in range(S)], dim=1)


def td_loss_grad(flat_params, flat_target, s_state, actions, rewards, s_next_state, gamma=0.99,
                 edge_index=None, edge_index_next=None, conv: str = "gat", dtype=torch.float32):
    """TD loss and its gradient (train_gcn_dqn.py:113-124) on S sampled graphs of N nodes.

    s_state / s_next_state: [S,N,4] (pos, vel); actions [S,N] int; rewards [S,N].
    conv="gcn": the a13 GCNConv variant (parity unpinned) on complete graphs, in dense form;
    conv="gcn_edges": the same in PyG's edge-list arithmetic (gcn_conv_edges); conv="gat_dense":
    the GAT in its dense multiplicity form (q_forward_dense) on complete graphs.  The alternate
    forms are the same math with every term formed and summed differently: further fp32
    evaluations for the tests' noise estimates.
    dtype=torch.float64 evaluates the same restatement in double precision from the same fp32
    inputs: the "exact" value both fp32 paths (this oracle and the GPU) are measured against.
    Returns (loss, flat grad [N_PARAMS], online Q at the taken actions, TD targets).
    """
    if conv in ("gcn", "gcn_edges", "gat_dense") and (edge_index is not None or edge_index_next is not None):
        # these restatements build complete graphs themselves: an edge list would be ignored and the
        # gradient (and any noise bound taken from it) would silently belong to the wrong graph
        raise ValueError(f"conv={conv!r} restates complete graphs only; edge_index must be None")
    if conv in ("gcn", "gcn_edges"):
        return _td_loss_grad_gcn(flat_params, flat_target, s_state, actions, rewards, s_next_state, gamma, dtype,
                                 edges=conv == "gcn_edges")
    if conv == "gat_dense":   # GCN.forward on the dense multiplicity form (q_forward_dense), complete graphs
        return _td_loss_grad_gat_dense(flat_params, flat_target, s_state, actions, rewards, s_next_state, gamma, dtype)
    S, N, _ = s_state.shape
    params = {k: v.to(dtype).clone().requires_grad_(True) for k, v in unflatten_params(flat_params).items()}
    tparams = {k: v.to(dtype) for k, v in unflatten_params(flat_target).items()}
    x = node_features(s_state[..., :2], s_state[..., 2:4]).reshape(S * N, N_FEATURES).to(dtype)
    xn = node_features(s_next_state[..., :2], s_next_state[..., 2:4]).reshape(S * N, N_FEATURES).to(dtype)
    ei = complete_batch_edge_index(S, N) if edge_index is None else edge_index
    ein = ei if edge_index_next is None else edge_index_next
    a = actions.reshape(-1).to(torch.long)
    r = rewards.reshape(-1).to(torch.float32).to(dtype)
    values = q_forward_edges(params, x, ei).gather(1, a.unsqueeze(1))
    with torch.no_grad():
        next_values = q_forward_edges(tparams, xn, ein).max(dim=1)[0]
    target = r + gamma * next_values
    loss = torch.nn.MSELoss()(values, target.unsqueeze(1))
    loss.backward()
    grad = torch.cat([params[k].grad.reshape(-1) for k, _ in PARAM_ORDER]).clone()
    return float(loss.item()), grad, values.detach().squeeze(1), target


def _td_loss_grad_gat_dense(flat_params, flat_target, s_state, actions, rewards, s_next_state, gamma,
                            dtype=torch.float32):
    S, N, _ = s_state.shape
    params = {k: v.to(dtype).clone().requires_grad_(True) for k, v in unflatten_params(flat_params).items()}
    tparams = {k: v.to(dtype) for k, v in unflatten_params(flat_target).items()}
    mult = multiplicity_complete(S, N).to(dtype)
    x = node_features(s_state[..., :2], s_state[..., 2:4]).to(dtype)
    xn = node_features(s_next_state[..., :2], s_next_state[..., 2:4]).to(dtype)
    a = actions.reshape(-1).to(torch.long)
    r = rewards.reshape(-1).to(torch.float32).to(dtype)
    values = q_forward_dense(params, x, mult).reshape(S * N, -1).gather(1, a.unsqueeze(1))
    with torch.no_grad():
        next_values = q_forward_dense(tparams, xn, mult).reshape(S * N, -1).max(dim=1)[0]
    target = r + gamma * next_values
    loss = torch.nn.MSELoss()(values, target.unsqueeze(1))
    loss.backward()
    grad = torch.cat([params[k].grad.reshape(-1) for k, _ in PARAM_ORDER]).clone()
    return float(loss.item()), grad, values.detach().squeeze(1), target


def _td_loss_grad_gcn(flat_params, flat_target, s_state, actions, rewards, s_next_state, gamma,
                      dtype=torch.float32, edges: bool = False):
    S, N, _ = s_state.shape
    params = {k: v.to(dtype).clone().requires_grad_(True) for k, v in unflatten_params(flat_params).items()}
    tparams = {k: v.to(dtype) for k, v in unflatten_params(flat_target).items()}
    mult = multiplicity_complete(S, N).to(dtype)
    x = node_features(s_state[..., :2], s_state[..., 2:4]).to(dtype)
    xn = node_features(s_next_state[..., :2], s_next_state[..., 2:4]).to(dtype)
    a = actions.reshape(-1).to(torch.long)
    r = rewards.reshape(-1).to(torch.float32).to(dtype)
    if edges:   # PyG's edge-list arithmetic on the Batch of complete graphs
        ei = complete_batch_edge_index(S, N)
        fwd = lambda p_, x_: gcn_conv_edges(p_, x_.reshape(S * N, -1), ei, S * N)  # noqa: E731
    else:
        fwd = lambda p_, x_: gcn_conv_dense(p_, x_, mult).reshape(S * N, -1)  # noqa: E731
    values = fwd(params, x).gather(1, a.unsqueeze(1))
    with torch.no_grad():
        next_values = fwd(tparams, xn).max(dim=1)[0]
    target = r + gamma * next_values
    loss = torch.nn.MSELoss()(values, target.unsqueeze(1))
    loss.backward()
    grad = torch.cat([(params[k].grad if params[k].grad is not None else torch.zeros_like(params[k])).reshape(-1)
                      for k, _ in PARAM_ORDER]).clone()
    return float(loss.item()), grad, values.detach().squeeze(1), target


@contextlib.contextmanager
def correctly_rounded_linears():
    """Inside this context every F.linear of the restatement (the GAT / GCN lin, lin1 and lin2, and
    autograd's products for them) is evaluated in float64 and rounded once to fp32: a further fp32
    evaluation of the same function that differs from torch's only in each dot product's rounding,
    i.e. in Q's last bits.  Test infrastructure: it measures how far a legitimate fp32 forward moves
    the gradient (tools/fwd_rounding.py), and it is the fifth member of the gradient bound's fp32
    spread (tests/test_gpu_parity_large.py oracle_grad_orders).  It replaces
    torch.nn.functional.linear process-wide while the context is open (restored on exit, also on an
    exception), so it is not for use beside other threads calling torch."""
    lin0 = F.linear

    def lin_cr(x, w, b=None):
        y = x.double() @ w.double().t()
        if b is not None:
            y = y + b.double()
        return y.to(x.dtype)

    F.linear = lin_cr
    try:
        yield
    finally:
        F.linear = lin0


def clip_adam(flat_params, grad, adam_m, adam_v, adam_step: int, lr=1e-3, betas=(0.9, 0.999), eps=1e-8,
              max_norm=1.0):
    """clip_grad_norm_(params, max_norm) + torch.optim.Adam step (train_gcn_dqn.py:85,125-126)
    with the gradient `grad` already in place.  Returns (params, m, v, total_norm)."""
    plist = [v.clone().requires_grad_(True) for v in unflatten_params(flat_params).values()]
    o = 0
    for p in plist:
        n = p.numel()
        p.grad = torch.as_tensor(grad[o:o + n], dtype=torch.float32).reshape(p.shape).clone()
        o += n
    total_norm = torch.nn.utils.clip_grad_norm_(plist, max_norm)
    opt = torch.optim.Adam(plist, lr=lr, betas=betas, eps=eps, foreach=False)
    if adam_step > 0:
        st = opt.state_dict()
        o = 0
        for i, p in enumerate(plist):
            n = p.numel()
            st["state"][i] = {
                "step": torch.tensor(float(adam_step)),
                "exp_avg": torch.as_tensor(adam_m[o:o + n], dtype=torch.float32).reshape(p.shape).clone(),
                "exp_avg_sq": torch.as_tensor(adam_v[o:o + n], dtype=torch.float32).reshape(p.shape).clone(),
            }
            o += n
        opt.load_state_dict(st)
    opt.step()
    st = opt.state_dict()["state"]
    m = torch.cat([st[i]["exp_avg"].reshape(-1) for i in range(len(plist))])
    v = torch.cat([st[i]["exp_avg_sq"].reshape(-1) for i in range(len(plist))])
    newp = torch.cat([p.detach().reshape(-1) for p in plist])
    return newp, m, v, float(total_norm)


def td_step(flat_params, flat_target, adam_m, adam_v, adam_step: int,
            s_state, actions, rewards, s_next_state, gamma=0.99, lr=1e-3,
            betas=(0.9, 0.999), eps=1e-8, max_norm=1.0, edge_index=None, edge_index_next=None, conv="gat"):
    """One DQN update (train_gcn_dqn.py:112-137): td_loss_grad + clip_adam.

    Returns dict(loss, grad (pre-clip), total_norm, params, m, v, step, values, target).
    """
    loss, grad, values, target = td_loss_grad(flat_params, flat_target, s_state, actions, rewards, s_next_state,
                                              gamma, edge_index, edge_index_next, conv)
    newp, m, v, total_norm = clip_adam(flat_params, grad, adam_m, adam_v, adam_step, lr, betas, eps, max_norm)
    return dict(loss=loss, grad=grad, total_norm=total_norm, params=newp,
                m=m, v=v, step=adam_step + 1, values=values, target=target)
