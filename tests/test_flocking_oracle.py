"""Flocking scenario (src/scenarios/flocking_scenario.py) in the oracle: the restatement
(``flocking_reward`` recomputes the goal term's "previous" value from the pre-step positions and
carries the spread's as explicit state, ``flocking_reset_spread`` after a reset) against a
stateful restatement that replays the scenario's own call sequence: the reset loop (:93-122,
agent i measured against the new positions of agents < i and the zeroed ones of agents > i)
and every reward call (:140-142, :163-164), over rollouts that start at a reset.
Parity unpinned against the reference itself: it records no Flocking trajectories."""
import math

import torch

from oracle import swarm_oracle as O


class _StatefulFlocking:
    """The scenario's reward() call sequence with its per-agent state (B envs at once;
    ``if agent.on_goal`` written as a where)."""

    def __init__(self, pos):
        """reset_world_at (:93-122) on states VMAS's World.reset has just zeroed: the loop sets
        agent i's position, then measures it against the current positions of all agents."""
        self.N = pos.shape[1]
        goal = O.f32(O.GOAL)
        cur = torch.zeros_like(pos)   # World.reset: every entity at the origin
        self.prev_goal, self.prev_agents = [], []
        for i in range(self.N):
            cur[:, i] = pos[:, i]                                   # agent.set_pos
            self.prev_goal.append(torch.linalg.vector_norm(cur[:, i] - goal, dim=1) * 10.0)
            self.prev_agents.append(self._spread(cur, i))

    def _spread(self, pos, i):
        d = torch.stack([torch.linalg.vector_norm(pos[:, i] - pos[:, j], dim=-1)
                         for j in range(self.N) if j != i], dim=1)
        return (d - 0.15).pow(2).mean(-1) * 10.0

    def reward(self, pos):
        goal = O.f32(O.GOAL)
        collective = 0
        for i in range(self.N):
            d = torch.linalg.vector_norm(pos[:, i] - goal, dim=-1)
            shaped = d * 10.0
            r = self.prev_goal[i] - shaped
            self.prev_goal[i] = shaped
            r = torch.where(d < 0.05, r + 50, r)
            avoid = torch.zeros(pos.shape[0])
            for j in range(self.N):
                if j != i:
                    gd = (torch.linalg.vector_norm(pos[:, i] - pos[:, j], dim=-1) - 0.05) - 0.05
                    avoid = avoid + torch.where(gd <= 0.005, -1.0, 0.0)
            now = self._spread(pos, i)
            dist_rew = self.prev_agents[i] - now
            self.prev_agents[i] = now
            collective = collective + ((r + avoid) + dist_rew)
        return collective


def _rollout(N, B, T, seed):
    g = torch.Generator().manual_seed(seed)
    c = O.reset_centres(O.SCENARIO_FLOCK, B, seed, 0, shared=False)
    pos = O.grid_positions(c, N)
    vel = torch.zeros(B, N, 2)
    ref = _StatefulFlocking(pos)
    spread = O.flocking_reset_spread(pos)
    assert torch.allclose(spread, torch.stack(ref.prev_agents, 1), rtol=0, atol=1e-4)
    for t in range(T):
        acts = torch.randint(0, 9, (B, N), generator=g)
        out = O.env_step(pos, vel, acts, O.SCENARIO_FLOCK, prev_spread=spread)
        want = ref.reward(out["pos"])
        assert torch.allclose(out["rew"][:, 0], want, rtol=0, atol=2e-5 * max(1.0, want.abs().max().item())), (N, t)
        assert torch.equal(out["rew"][:, 0], out["rew"][:, -1])
        if t > 0:   # later steps: the stored spread is the pre-step positions' own (recomputable)
            assert torch.equal(O.env_step(pos, vel, acts, O.SCENARIO_FLOCK)["rew"], out["rew"])
        pos, vel, spread = out["pos"], out["vel"], out["spread"]
    return out


def test_reward_with_carried_spread_equals_stateful_scenario():
    for N, B, T in ((2, 16, 30), (5, 32, 40), (8, 16, 25), (12, 8, 15)):
        _rollout(N, B, T, seed=N)


def test_first_step_after_reset_uses_the_reset_loop_spread():
    """the reset loop measures agent i against agents j > i still at the origin, so
    the first step's spread term differs from one recomputed on the reset grid.  N = 10 at the
    mean centre (-1.6, 1.6): the collective reward is ~+215 higher than the recomputed one."""
    N = 10
    pos = O.grid_positions(torch.tensor([[-1.6, 1.6]]), N)
    vel = torch.zeros(1, N, 2)
    acts = torch.zeros(1, N, dtype=torch.long)
    ref = _StatefulFlocking(pos)
    first = O.env_step(pos, vel, acts, O.SCENARIO_FLOCK, prev_spread=O.flocking_reset_spread(pos))
    naive = O.env_step(pos, vel, acts, O.SCENARIO_FLOCK)
    want = ref.reward(first["pos"])
    assert abs(first["rew"][0, 0].item() - want.item()) <= 1e-4 * abs(want.item())
    gap = first["rew"][0, 0].item() - naive["rew"][0, 0].item()
    assert 150.0 < gap < 300.0, gap
    # agent 0 sees only zeroed partners; the last agent sees the whole new grid
    assert torch.allclose(O.flocking_reset_spread(pos)[:, -1], O._flock_agent_spread(pos, N - 1))


def test_goal_bonus_and_contacts():
    # two agents: one sitting on the goal, the other touching it (|d| = 0.1 <= 0.105)
    goal = O.f32(O.GOAL)
    pos = torch.stack([goal, goal + torch.tensor([0.1, 0.0])])[None]
    vel = torch.zeros(1, 2, 2)
    out = O.env_step(pos, vel, torch.zeros(1, 2, dtype=torch.long), O.SCENARIO_FLOCK)
    assert out["hits"].item() == 2.0                         # one contact, counted by each agent
    # goal bonus for agent 0 only; contacts -1 each; positions change by the collision force
    assert out["rew"][0, 0].item() > 40.0


def test_reset_centre_distribution():
    c = O.reset_centres(O.SCENARIO_FLOCK, 4096, 3, 0, shared=False)
    mean = c.double().mean(0)
    assert math.isclose(mean[0].item(), -1.6, abs_tol=0.03) and math.isclose(mean[1].item(), 1.6, abs_tol=0.03)
    assert math.isclose(c.double().std(0)[0].item(), 0.4, abs_tol=0.03)


# ---------------------------------------------------------------- the Flocking checkpoints' GAT3
def test_gat3_dense_equals_edge_list(golden_weights):
    for seed, N, graph in ((0, 2, O.GRAPH_COMPLETE), (3, 5, O.GRAPH_KNN), (7, 8, O.GRAPH_COMPLETE),
                           (9, 12, O.GRAPH_KNN)):
        P = O.gat3_unflatten(golden_weights["flocking_gat3"][seed])
        g = torch.Generator().manual_seed(seed)
        pos, vel = torch.randn(6, N, 2, generator=g) * 0.4, torch.randn(6, N, 2, generator=g) * 0.2
        x = O.node_features(pos, vel)
        mult = O.graph_multiplicity(pos, graph, k=min(5, N))
        q_dense = O.gat3_q_forward_dense(P, x, mult)
        q_edges = O.gat3_q_forward_edges(P, x.reshape(-1, 7), O.edge_index_from_multiplicity(mult))
        assert torch.allclose(q_dense.reshape(-1, 9), q_edges, rtol=1e-5, atol=1e-5)


def test_gat3_host_layout_matches_the_checkpoints(golden_weights):
    import swarm_amd
    from swarm_amd.engine import PARAM_ORDER_GAT3, flatten_state_dict, unflatten_params
    assert PARAM_ORDER_GAT3 == O.GAT3_PARAM_ORDER and O.GAT3_N_PARAMS == 409
    flat = torch.tensor(golden_weights["flocking_gat3"][4])
    sd = unflatten_params(flat, "gat3")
    m = swarm_amd.GCN.from_state_dict(sd)
    assert m.layers == 3 and m.net == "gat3"
    assert torch.equal(m.flat_params("cpu"), flat) and torch.equal(flatten_state_dict(sd, net="gat3"), flat)
    assert list(m.state_dict()) == [k for k, _ in O.GAT3_PARAM_ORDER]   # the .pth key order
