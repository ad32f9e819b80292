"""Pin the CPU oracle to the reference's own recorded outputs (no GPU).

Fixtures (tests/golden/, made by tests/golden/make_golden.py from
/root/reference/data): trained weights and recorded evaluation trajectories of
src/simulation/simulator.py (kNN k=5).  For every recorded tick the
oracle rebuilds the observation (recorded positions + velocities derived from
them), the kNN graph, the GAT Q-values and the argmax, and must reproduce the
action the reference took (derived from the recorded next positions); it must
also reproduce the recorded per-tick distance/hits and per-episode result.csv.
"""
import numpy as np
import pytest
import torch

from oracle import swarm_oracle as O
from tests.conftest import RECORDED_AGENTS, record

CASES = [(scen, sid, seed, n) for scen, sid in (("go_to", O.SCENARIO_GOTO), ("obstacle_avoidance", O.SCENARIO_OA))
         for seed in (0, 4) for n in RECORDED_AGENTS]


def _weights(golden_weights, scen, seed):
    return O.unflatten_params(torch.tensor(golden_weights[scen][seed]))


@pytest.mark.parametrize("scen,sid,seed,n", CASES)
def test_oracle_reproduces_recorded_actions(golden_weights, trajectories, scen, sid, seed, n):
    params = _weights(golden_weights, scen, seed)
    total = match = 0
    for ep in range(8):
        key = f"{scen}/s{seed}/n{n}/e{ep}"
        P = trajectories[key + "/pos"]                       # [T,N,2] fp32 recorded
        ref = trajectories[key + "/ref_action"]
        T = P.shape[0]
        P64 = P.astype(np.float64)
        V = np.zeros_like(P64)
        V[1:] = (P64[1:] - P64[:-1]) / 0.1
        pos = torch.tensor(P[1:T - 1])
        vel = torch.tensor(V[1:T - 1].astype(np.float32))
        x = O.node_features(pos, vel)
        mult = O.multiplicity_knn(O.knn_sets(pos, 5))
        q = O.q_forward_dense(params, x, mult)
        act = O.argmax_first(q).numpy()
        r = ref[1:T - 1]
        ok = act == r
        qs = q.sort(dim=-1, descending=True).values
        gap = (qs[..., 0] - qs[..., 1]).numpy()
        # misses allowed only at argmax near-ties (recorded velocities are derived, ~1e-6 noise)
        assert np.all(gap[~ok] < 1e-4), f"{key}: clear-margin action mismatch"
        total += ok.size
        match += ok.sum()
    assert match / total >= 0.999


@pytest.mark.parametrize("scen,sid,seed,n", CASES)
def test_oracle_env_step_matches_recorded_positions(trajectories, scen, sid, seed, n):
    for ep in range(2):
        key = f"{scen}/s{seed}/n{n}/e{ep}"
        P = trajectories[key + "/pos"]
        ref = trajectories[key + "/ref_action"]
        P64 = P.astype(np.float64)
        V = np.zeros_like(P64)
        V[1:] = (P64[1:] - P64[:-1]) / 0.1
        T = P.shape[0]
        pos = torch.tensor(P[1:T - 1])
        vel = torch.tensor(V[1:T - 1].astype(np.float32))
        a = torch.tensor(ref[1:T - 1].astype(np.int64))
        st = O.env_step(pos, vel, a, sid)
        err = (st["pos"].double().numpy() - P64[2:T]).__abs__().max()
        assert err < 2e-6, err


@pytest.mark.parametrize("scen,sid,seed,n", CASES)
def test_oracle_metrics_match_recorded(trajectories, scen, sid, seed, n):
    res = trajectories[f"{scen}/s{seed}/n{n}/result"]
    for ep in range(8):
        key = f"{scen}/s{seed}/n{n}/e{ep}"
        P = torch.tensor(trajectories[key + "/pos"])
        dist_goal = O.vector_norm2(P - O.f32(O.GOAL))                     # [T,N]
        avg = torch.mean(dist_goal, dim=1).double().numpy()
        np.testing.assert_allclose(avg, trajectories[key + "/dist"], atol=1e-6)
        if sid == O.SCENARIO_OA:
            d_obs = (O.vector_norm2(P - O.f32(O.OBSTACLE)) - O.SPHERE_RADIUS) - O.SPHERE_RADIUS
            hits = (d_obs <= 0.2).sum(dim=1).double().numpy()
            np.testing.assert_array_equal(hits, trajectories[key + "/hits"])
            obst = torch.where(d_obs <= 1, -(1 - d_obs), torch.tensor(0.0))
            rew = (-dist_goal + 2.5 * obst).sum(dim=1)
        else:
            rew = (-dist_goal).sum(dim=1) * P.shape[1]    # collective reward, identical for every agent
        T = P.shape[0]
        row = res[ep]
        assert abs(rew.double().sum().item() / T - row[1]) <= 1e-4 * max(1.0, abs(row[1]))
        assert abs(avg[-1] - row[3]) < 1e-6 and abs(avg[0] - row[4]) < 1e-6
        assert trajectories[key + "/hits"].sum() == row[2]


def _recorded_action(pos, vel, p_next, sid):
    """The action the recorded run took from (pos, vel) [N, 2] to reach p_next: u = ((p_next - pos)
    / dt - 0.75 vel) / dt - f_coll(pos), rounded to the levels {-1, 0, 1}."""
    f = O.env_step(pos[None], vel[None], torch.zeros(1, pos.shape[0], dtype=torch.long), sid)["force"][0].double()
    u = ((torch.as_tensor(p_next).double() - pos.double()) / 0.1 - 0.75 * vel.double()) / 0.1 - f
    ur = u.round()
    assert (u - ur).abs().max() < 1e-2 and ur.abs().max() <= 1
    lidx = {0.0: 0, -1.0: 1, 1.0: 2}
    return torch.tensor([3 * lidx[float(x)] + lidx[float(y)] for x, y in ur.tolist()])


@pytest.mark.parametrize("scen,sid,seed,n", CASES)
def test_oracle_closed_loop_reproduces_recorded_episodes(golden_weights, trajectories, scen, sid, seed, n):
    """Whole evaluation episodes, closed loop (VERDICT r3 "next" #8): each of the 8 recorded
    episodes starts from its reset formation, recovered from the first two recorded steps
    (O.reset_from_first_step), and the oracle then runs the reference's loop on its own state
    (simulator.py:59-84: kNN-5 graph -> GCN.forward -> argmax -> env.step) for max_steps ticks.
    An episode either reproduces every recorded tick bit for bit, and then its result.csv row
    (Reward, Collisions, Distance end / beginning) bit for bit too (the reward accumulated in fp32
    in the reference's order, O.episode_result), or it leaves the record at a tick where the
    oracle's action differs from the recorded one only inside the 1e-4 argmax tie band of SURVEY
    §8(c)(ii).  Over the 128 recorded episodes of N = 5..12 exactly one leaves (OA, model seed 4,
    7 agents, episode 0, tick 71: agent 6's Q for actions 3 and 2 are one fp32 ulp apart at
    |Q| = 204, the float64 evaluation prefers the recorded 2 by 2.9e-6, and every fp32 formulation
    here, dense and PyG edge-list, rounds to 3)."""
    params = _weights(golden_weights, scen, seed)
    res = trajectories[f"{scen}/s{seed}/n{n}/result"]
    P = np.stack([trajectories[f"{scen}/s{seed}/n{n}/e{e}/pos"] for e in range(8)])   # [8, T, N, 2]
    T = P.shape[1]
    pos = torch.stack([O.reset_from_first_step(P[e, 0], P[e, 1], sid)[0] for e in range(8)])
    vel = torch.zeros(8, n, 2)
    on = [True] * 8          # episode still on its recorded trajectory
    left = []
    rews, avgs, hits = [], [], []
    for t in range(T):
        out = O.act_tick(params, pos, vel, sid, O.GRAPH_KNN, 5, 0.0, 0, t)
        for e in range(8):
            if on[e] and not torch.equal(out.step["pos"][e], torch.tensor(P[e, t])):
                a_ref = _recorded_action(pos[e], vel[e], P[e, t], sid)
                a_or = out.actions[e]
                diff = a_or != a_ref
                assert bool(diff.any()), (e, t, "left the recorded trajectory without an action change")
                q = out.q[e].double()
                gap = (q[torch.arange(n), a_or] - q[torch.arange(n), a_ref])[diff]
                assert bool((gap.abs() <= 1e-4).all()), (e, t, gap)
                on[e] = False
                left.append((e, t, float(gap.abs().max())))
        pos, vel = out.step["pos"], out.step["vel"]
        rews.append(out.step["rew"])
        avgs.append(out.step["avg_dist"])
        hits.append(out.step["hits"])
    rews, avgs, hits = torch.stack(rews, 1), torch.stack(avgs, 1), torch.stack(hits, 1)
    record(f"oracle closed loop {scen} seed {seed} N={n}", {"bitwise": sum(on), "left_after_near_tie": len(left),
                                                              "left": left})
    assert sum(on) >= 7, left
    for e in range(8):
        if on[e]:
            got = O.episode_result(rews[e], avgs[e], hits[e])
            assert got == tuple(res[e, 1:]), (e, got, res[e])
