"""The acting half against the oracle at the benchmarked sizes (VERDICT r3 "next" #2).

C2 = GoTo, 8 agents x 1024 envs, GAT; C3 = ObstacleAvoidance, 12 agents x 1024 envs, GAT;
C5's shard = ObstacleAvoidance, 5 and 12 agents x 512 envs per GPU, GAT and the a13 GCNConv
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
