"""The acting half against the oracle at the benchmarked sizes (VERDICT r3 "next" #2).

C2 = GoTo, 8 agents x 1024 envs, GAT; C3 = ObstacleAvoidance, 12 agents x 1024 envs, GAT;
C5's shard = ObstacleAvoidance, every N of the 5-12 sweep x 512 envs per GPU, GAT and the a13 GCNConv
variant.  The fused training tick (swarm_train_tick + swarm_reduce_advance, the bench's launch) runs
from a reset formation for four ticks with eps = 0.3, and every tick is compared with the oracle's
act_tick (train_gcn_dqn.py:161-172: complete graph -> GCN.forward -> eps-greedy -> env.step), on the
state the tick started from and the weights the tick acted with (the previous tick's deferred clip +
Adam step applied in the launch's prologue, read back from the learner's current row):
- the reset formation (go_to_position_scenario.py:83-106 / obstacle_avoidance_scenario.py:94-133);
- Q of every agent of every env within Q_ULP fp32 ulps of max(|Q|, 1) and 1e-5 relative;
- actions equal wherever the oracle's top-2 gap exceeds 1e-4 or the env explored (every env's
  coin and random draws are Philox-keyed, so exploring envs match exactly);
- env.step on the GPU's actions: positions and velocities within 1e-6 (positions bit-exact for
  agents with no contact force), rewards within 1e-6 relative, obstacle hits equal, mean goal
  distance within 1e-6 relative;
- the replay push of the tick's slot: s, a bit-exact, r and s' equal to the tick's outputs.
"""
import pytest
import torch

from oracle import swarm_oracle as O
from tests.conftest import assert_close_rel, assert_close_ulp, error_stats, record
from tests.test_gpu_parity import Q_ULP, _tie_mask

pytestmark = pytest.mark.gpu

CASES = [("C2", "GoTo", 8, 1024, "gat"), ("C3", "ObstacleAvoidance", 12, 1024, "gat"),
         ("C5 N=5 GAT", "ObstacleAvoidance", 5, 512, "gat"), ("C5 N=12 GAT", "ObstacleAvoidance", 12, 512, "gat"),
         ("C5 N=5 GCN", "ObstacleAvoidance", 5, 512, "gcn"), ("C5 N=12 GCN", "ObstacleAvoidance", 12, 512, "gcn")]
# C5's sweep interior (VERDICT r5 "next" #1): every agent count from 5 to 12, GAT and GCN
CASES += [(f"C5 N={n} {conv.upper()}", "ObstacleAvoidance", n, 512, conv) for n in (6, 7, 8, 9, 10, 11) for conv in ("gat", "gcn")]
# the GCN variant (a13) at C2's and C3's full 1,024-env shapes too (the sweep's "C2 GCN train" line)
CASES += [("C2 GCN", "GoTo", 8, 1024, "gcn"), ("C3 GCN", "ObstacleAvoidance", 12, 1024, "gcn")]
SCEN = {"GoTo": O.SCENARIO_GOTO, "ObstacleAvoidance": O.SCENARIO_OA}
EPS, SEED = 0.3, 21


@pytest.fixture(scope="module")
def sw():
    import swarm_amd
    swarm_amd.load_library()
    return swarm_amd


@pytest.mark.parametrize("name,scen,N,B,conv", CASES)
def test_fused_tick_acting_half_at_benchmark_size(sw, golden_weights, name, scen, N, B, conv):
    key = "go_to" if scen == "GoTo" else "obstacle_avoidance"
    p = torch.tensor(golden_weights[key][3])
    eng = sw.SwarmEngine(scen, N, B, seed=SEED, params=p, batch=B, replay_capacity=6 * B, eps=EPS, conv=conv,
                         update_target_every=100000)
    assert eng.fused
    # two pushed slots first, so that the first fused tick trains (its TD batch needs B graphs)
    eng.reset(0)
    for _ in range(2):
        eng.act(push=True, full_out=False)
        eng.advance()
    eng.reset(1)   # episode 1: the reset the fused ticks start from
    torch.cuda.synchronize()
    ref_pos = O.grid_positions(O.reset_centres(SCEN[scen], B, SEED, 1, False, random_oa=True), N)
    st = eng.state.cpu()
    record(f"{name} reset positions", error_stats(st[..., :2], ref_pos))
    assert (st[..., :2] - ref_pos).abs().max() < 2e-6 and not st[..., 2:].any()
    n_tie = 0
    for t in range(4):
        c = eng.read_ctrl()
        pos, vel = eng.state.cpu()[..., :2].clone(), eng.state.cpu()[..., 2:].clone()
        eng.train_tick(full_out=True)
        torch.cuda.synchronize()
        assert eng.handoff_errors() == 0
        w_used = eng.params.cpu().clone()
        ref = O.act_tick(O.unflatten_params(w_used), pos, vel, SCEN[scen], O.GRAPH_COMPLETE, 0, EPS, SEED, c["tick"],
                         conv=conv)
        assert_close_ulp(eng.q.cpu(), ref.q, Q_ULP, f"{name} tick {t} Q", scale=1.0, rel_floor=1e-5)
        acts = eng.actions.cpu().long()
        clear = _tie_mask(ref.q) | ref.explore[:, None]
        assert ref.explore.any() and (~ref.explore).any()
        assert torch.equal(acts[clear], ref.actions[clear]), f"{name} tick {t}: action outside the tie band"
        n_tie += int((~clear).sum())
        # env.step on the actions the GPU took (tie-band agents included)
        step = O.env_step(pos, vel, acts, SCEN[scen])
        st = eng.state.cpu()
        record(f"{name} tick {t} s'", error_stats(st, torch.cat([step["pos"], step["vel"]], -1)))
        assert (st[..., :2] - step["pos"]).abs().max() <= 1e-6 and (st[..., 2:] - step["vel"]).abs().max() <= 1e-6
        free = step["force"].eq(O.decode_actions(acts)).all(-1)
        assert torch.equal(st[..., :2][free], step["pos"][free])
        assert_close_rel(eng.reward.cpu(), step["rew"], 1e-6, f"{name} tick {t} reward")
        assert_close_rel(eng.avg_dist.cpu(), step["avg_dist"], 1e-6, f"{name} tick {t} avg distance")
        assert torch.equal(eng.hits.cpu(), step["hits"])
        # the replay push of this tick's slot
        ws = c["write_slot"]
        assert torch.equal(eng.rep_s[ws].cpu(), torch.cat([pos, vel], -1))
        assert torch.equal(eng.rep_a[ws].cpu().long(), acts)
        assert torch.equal(eng.rep_r[ws].cpu(), eng.reward.cpu())
        assert torch.equal(eng.rep_s1[ws].cpu(), st)
    record(f"{name}: agents in the 1e-4 tie band over 4 ticks", {"n": n_tie, "of": 4 * B * N})
    assert eng.read_ctrl()["adam_step"] >= 2   # the weights changed between the compared ticks


# ------------------------------------------------------------------ kNN acting at benchmark size
# VERDICT r4 "next" #5: the reference's EVALUATION graph is kNN (simulator.py:15-24, k = 10; the
# recorded 5/8-agent evaluations ran k = 5), and the sweep's acting lines run it at 1,024 envs:
# OA 12 x 1024 kNN-10 and GoTo 8 x 1024 kNN-5.  Both halves of the acting path on that graph:
# (1) single acting ticks (swarm_act_step, kNN built every tick, tie path without memo) against
#     O.act_tick on the state each tick started from: neighbour sets / edge multiplicities
#     bit-exact (the tie-heavy reset grid included), Q, actions outside the tie band, s', rewards,
#     hits;
# (2) the rollout launch (swarm_rollout: kNN + GAT specialised kernel, state in registers across
#     ticks, the tie memo) against the oracle's own closed loop (kNN -> GCN.forward -> argmax ->
#     env.step, simulator.py:59-68) from the same reset: every env whose oracle Q never had a
#     top-2 gap inside the 1e-4 tie band follows the oracle's trajectory (positions, mean goal
#     distance and hits of every tick).
KNN_CASES = [("OA 12x1024 kNN-10", "ObstacleAvoidance", 12, 1024, 10), ("GoTo 8x1024 kNN-5", "GoTo", 8, 1024, 5)]


@pytest.mark.parametrize("name,scen,N,B,k", KNN_CASES)
def test_knn_acting_ticks_at_benchmark_size(sw, golden_weights, name, scen, N, B, k):
    key = "go_to" if scen == "GoTo" else "obstacle_avoidance"
    p = torch.tensor(golden_weights[key][0])
    eng = sw.SwarmEngine(scen, N, B, seed=SEED, params=p, graph="knn", knn_k=k, eps=EPS, learn=False)
    mult = torch.zeros(B * N * N, dtype=torch.uint8, device="cuda")
    eng.out.mult = mult.data_ptr()
    eng.reset(0)
    n_tie = 0
    for t in range(4):
        pos, vel = eng.state.cpu()[..., :2].clone(), eng.state.cpu()[..., 2:].clone()
        eng.ctrl[0] = t   # the tick keys the eps coin and the random actions
        eng.act(push=False)
        torch.cuda.synchronize()
        ref = O.act_tick(O.unflatten_params(p), pos, vel, SCEN[scen], O.GRAPH_KNN, k, EPS, SEED, t)
        assert torch.equal(mult.view(B, N, N).cpu().float(), ref.mult), f"{name} tick {t}: kNN multiplicities"
        assert_close_ulp(eng.q.cpu(), ref.q, Q_ULP, f"{name} tick {t} Q", scale=1.0, rel_floor=1e-5)
        acts = eng.actions.cpu().long()
        clear = _tie_mask(ref.q) | ref.explore[:, None]
        assert torch.equal(acts[clear], ref.actions[clear]), f"{name} tick {t}: action outside the tie band"
        n_tie += int((~clear).sum())
        step = O.env_step(pos, vel, acts, SCEN[scen])
        st = eng.state.cpu()
        record(f"{name} tick {t} s'", error_stats(st, torch.cat([step["pos"], step["vel"]], -1)))
        assert (st[..., :2] - step["pos"]).abs().max() <= 1e-6 and (st[..., 2:] - step["vel"]).abs().max() <= 1e-6
        assert_close_rel(eng.reward.cpu(), step["rew"], 1e-6, f"{name} tick {t} reward")
        assert torch.equal(eng.hits.cpu(), step["hits"])
    record(f"{name}: agents in the 1e-4 tie band over 4 kNN ticks", {"n": n_tie, "of": 4 * B * N})


@pytest.mark.parametrize("name,scen,N,B,k", KNN_CASES)
def test_knn_rollout_follows_the_oracle_closed_loop(sw, golden_weights, name, scen, N, B, k):
    T = 10
    key = "go_to" if scen == "GoTo" else "obstacle_avoidance"
    p = torch.tensor(golden_weights[key][0])
    eng = sw.SwarmEngine(scen, N, B, seed=SEED, params=p, graph="knn", knn_k=k, eps=0.0, learn=False)
    eng.reset(0)
    torch.cuda.synchronize()
    pos, vel = eng.state.cpu()[..., :2].clone(), eng.state.cpu()[..., 2:].clone()
    r = eng.rollout(T, tick0=0, eps=0.0, traj=True)
    torch.cuda.synchronize()
    tp, td, th = r["traj_pos"].cpu(), r["traj_dist"].cpu(), r["traj_hits"].cpu()
    params = O.unflatten_params(p)
    on = torch.ones(B, dtype=torch.bool)   # envs still on a trajectory the oracle pins
    worst = 0.0
    for t in range(T):
        ref = O.act_tick(params, pos, vel, SCEN[scen], O.GRAPH_KNN, k, 0.0, SEED, t)
        on &= ~(~_tie_mask(ref.q)).any(-1)   # an env leaves the comparison at its first tie-band tick
        pos, vel = ref.step["pos"], ref.step["vel"]
        e = (tp[t][on] - pos[on]).abs().max().item() if on.any() else 0.0
        worst = max(worst, e)
        assert e <= 1e-5, f"{name} tick {t}: rollout positions {e:.3e} from the oracle's closed loop"
        assert_close_rel(td[t][on], ref.step["avg_dist"][on], 1e-6, f"{name} rollout tick {t} mean goal distance")
        assert torch.equal(th[t][on], ref.step["hits"][on])
    record(f"{name} rollout vs oracle closed loop", {"max_abs": worst, "envs_compared_all_ticks": int(on.sum()),
                                                      "of": B, "ticks": T})
    assert int(on.sum()) >= B // 2, f"{name}: too few envs outside the tie band to compare ({int(on.sum())})"
