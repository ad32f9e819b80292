"""The learning half against the oracle at the BASELINE.json sizes (VERDICT r2 "next" #1, r3 #2/#7).

C2 = GoTo, 8 agents x 1024 envs, TD batch S = 1024 graphs (256 TD blocks, 256 gradient slabs
summed by the 105-block reduce); C3 = ObstacleAvoidance, 12 agents x 1024 envs, S = 1024 (one
graph per TD wave); C5's shard = ObstacleAvoidance, every N of the 5-12 sweep x 512 envs per GPU, S = 512,
GAT and the a13 GCNConv variant.  Both the reference-shaped API sequence (swarm_td_grad ->
swarm_grad_reduce -> swarm_adam_step, train_gcn_dqn.py:112-137) and the headline's fused
swarm_train_tick (whose TD graphs partly come from the tick's own replay slot through the
hand-off records) are compared with the oracle's autograd restatement (oracle.swarm_oracle
td_loss_grad / clip_adam), with replay content from real acting ticks (reset grid, collisions).

The sampled rows are not taken on trust: s' and r of every sampled transition are re-derived from
(s, a) by the oracle's env_step (simulator.py:59-68 / train_gcn_dqn.py:168-172 semantics), checked
against the GPU's ring, and the oracle's TD runs on the oracle's own s' and r.

Tolerances (fixed before the round-4 measurements; the achieved errors go to
parity_errors.gpu.json via conftest.record and are kept under profiles/):
- gradient, per parameter tensor: the GPU's largest distance to the float64 evaluation is at most
  4x the fp32 oracle's own plus 4 ulps of the tensor's largest element;
- the fp32 oracle's own error: the largest distance to float64 of five fp32 evaluations of the
  same sum (the batch in three orders, the other formulation: GAT dense / GCN edge-list, and every
  linear layer correctly rounded).  Round 6 added the fifth: the first four share torch's rounding
  of each per-node Q, which the TD error amplifies, and the correctly rounded evaluation itself
  landed at up to 10.5x their spread (C3 GCN's API update, where the GPU was at 6.0x and at 0.57 of
  the five-evaluation spread), so a bound of 4x the four-evaluation spread rejected a more accurate
  fp32 evaluation; both ratios are recorded per case (_record_forward_rounding);
- gradient, per element: within 1e-4 of the element's magnitude plus 2e-6 of the tensor's largest
  element (the pre-round-3 bound; round 3 had doubled it to admit a summation-order change, and
  that doubling is withdrawn) plus 4x the fp32 oracle's own distance to float64 on that very
  element (largest over the four evaluations).  The last term matters only where the TD error
  delta = Q - y cancels most of Q (small gradients: C5's first fused tick, the a13 variant at
  12 agents): there every fp32 evaluation's gradient error is set by Q's last bits, and the fp32
  oracle itself exceeds the pre-round-3 bound (3.6x on conv1.lin.weight at C5's first fused
  tick); both ratios are recorded;
- Adam, isolated from the gradient: m, v and the weights against torch.optim.Adam applied to the
  GPU's OWN gradient: m within 8 ulps and v within 16 ulps of the magnitude of their update terms
  (beta * old + (1 - beta) * new), the weights within 4 ulps of max(|w|, lr);
- end to end, weights after Adam within 2e-6 of torch's update on the fp32 oracle's gradient, plus,
  per element, the difference Adam itself makes of the two gradients' difference (round 6: near
  Adam's eps the update amplifies last-bit gradient differences; _end_to_end_weights).
"""
import pytest
import torch

from oracle import swarm_oracle as O
from tests.conftest import assert_close_rel, error_stats, fp32_ulp, record

pytestmark = pytest.mark.gpu

CASES = [("C2", "GoTo", 8, 1024, 1024, "gat"), ("C3", "ObstacleAvoidance", 12, 1024, 1024, "gat"),
         ("C5 N=5 GAT", "ObstacleAvoidance", 5, 512, 512, "gat"), ("C5 N=12 GAT", "ObstacleAvoidance", 12, 512, 512, "gat"),
         ("C5 N=5 GCN", "ObstacleAvoidance", 5, 512, 512, "gcn"), ("C5 N=12 GCN", "ObstacleAvoidance", 12, 512, 512, "gcn")]
# C5's sweep interior (VERDICT r5 "next" #1): N = 6, 7, 8 run the 8-slot kernels with 2 / 1 / 0 padded
# slots, N = 9, 10, 11 the 16-slot kernels with 7 / 6 / 5 padded slots (N = 12 has 4)
CASES += [(f"C5 N={n} {conv.upper()}", "ObstacleAvoidance", n, 512, 512, conv)
          for n in (6, 7, 8, 9, 10, 11) for conv in ("gat", "gcn")]
# the GCN variant (a13) at C2's and C3's full shapes (S = 1,024 graphs: 256 / 512 slabs)
CASES += [("C2 GCN", "GoTo", 8, 1024, 1024, "gcn"), ("C3 GCN", "ObstacleAvoidance", 12, 1024, 1024, "gcn")]
SCEN = {"GoTo": O.SCENARIO_GOTO, "ObstacleAvoidance": O.SCENARIO_OA}


@pytest.fixture(scope="module")
def sw():
    import swarm_amd
    swarm_amd.load_library()
    return swarm_amd


def _weights(golden_weights, scen, seed):
    key = "go_to" if scen == "GoTo" else "obstacle_avoidance"
    return torch.tensor(golden_weights[key][seed])


def _prefill(eng, slots):
    """slots acting ticks (eps-greedy, replay push, no learning) from a reset formation."""
    eng.reset(0)
    for _ in range(slots):
        eng.act(push=True, full_out=False)
        eng.advance()
    torch.cuda.synchronize()


def _rows(eng, idx, scen, name):
    """The sampled transitions (s, a, r, s'): s and a from the ring; s' and r re-derived from them
    by the oracle's env_step and checked against the ring (positions / velocities within 1e-6,
    positions bit-exact for agents with no contact force; reward within 1e-6 relative)."""
    B = eng.B
    idx = idx.cpu().long()
    slot, env = idx // B, idx % B
    s, a = eng.rep_s.cpu()[slot, env], eng.rep_a.cpu()[slot, env].long()
    r_gpu, s1_gpu = eng.rep_r.cpu()[slot, env], eng.rep_s1.cpu()[slot, env]
    step = O.env_step(s[..., :2], s[..., 2:], a, SCEN[scen])
    s1 = torch.cat([step["pos"], step["vel"]], -1)
    record(f"{name} ring s' vs oracle env_step", error_stats(s1_gpu, s1))
    assert (s1_gpu - s1).abs().max() <= 1e-6
    free = step["force"].eq(O.decode_actions(a)).all(-1)
    assert torch.equal(s1_gpu[..., :2][free], s1[..., :2][free])
    assert_close_rel(r_gpu, step["rew"], 1e-6, f"{name} ring r vs oracle env_step")
    return s, a, step["rew"].to(torch.float32), s1


def oracle_grad_orders(p, t, s, a, r, s1, conv="gat", seed=0, edge_fn=None):
    """The fp32 oracle's gradient evaluated five ways, each a valid fp32 evaluation of the same
    sum: the batch in three orders (as given, reversed, shuffled), on complete graphs the other
    formulation (GAT: the dense multiplicity form; GCN: PyG's edge-list arithmetic), whose terms are
    themselves formed differently, and every linear layer correctly rounded (the last entry); and
    the float64 value.  The first is the oracle.
    edge_fn(s_graphs) -> Batch edge_index for kNN / radius graphs (None: complete)."""
    S = s.shape[0]
    perms = [torch.arange(S), torch.arange(S - 1, -1, -1), torch.randperm(S, generator=torch.Generator().manual_seed(seed))]
    g32s, loss32 = [], None
    for q in perms:
        ei = None if edge_fn is None else edge_fn(s[q])
        ein = None if edge_fn is None else edge_fn(s1[q])
        loss, g, _, _ = O.td_loss_grad(p, t, s[q], a[q], r[q], s1[q], edge_index=ei, edge_index_next=ein, conv=conv)
        g32s.append(g)
        loss32 = loss if loss32 is None else loss32
    if edge_fn is None:   # complete graphs: the other formulation
        g32s.append(O.td_loss_grad(p, t, s, a, r, s1, conv="gcn_edges" if conv == "gcn" else "gat_dense")[1])
    ei = None if edge_fn is None else edge_fn(s)
    ein = None if edge_fn is None else edge_fn(s1)
    # and (round 6) every linear layer correctly rounded: differs from the others in Q's last bits,
    # which the three batch orders share (module docstring); always the LAST entry
    with O.correctly_rounded_linears():
        g32s.append(O.td_loss_grad(p, t, s, a, r, s1, edge_index=ei, edge_index_next=ein, conv=conv)[1])
    loss64, g64, _, _ = O.td_loss_grad(p, t, s, a, r, s1, edge_index=ei, edge_index_next=ein, conv=conv,
                                       dtype=torch.float64)
    return loss32, g32s, loss64, g64


def _grad_bound_check(name, g_gpu, g32s, g64):
    """Gradient vs the float64 evaluation (module docstring).  Gradient elements are sums over S*N
    nodes whose terms cancel, so an element's rounding error scales with its terms, not with its
    value: both fp32 paths sit thousands of ulps of the value away on such elements, and an ulp
    bound on the value alone would only test which summation order got luckier."""
    if torch.is_tensor(g32s):
        g32s = [g32s]
    o = 0
    worst_ratio_t, worst_elem, worst_k = 0.0, 0.0, None
    for k, shape in O.PARAM_ORDER:
        n = 1
        for s in shape:
            n *= s
        a, b = g_gpu[o:o + n].double(), g64[o:o + n]
        cs = [g[o:o + n].double() for g in g32s]
        gmax = float(b.abs().max())
        floor = 2e-6 * gmax
        st_gpu = error_stats(a, b, scale=floor)
        st_o32 = error_stats(cs[0], b, scale=floor)
        # per tensor: 4x the fp32 oracle's own largest distance + 4 ulps of the largest element
        o32_max = max(float((c - b).abs().max()) for c in cs)
        bound = 4.0 * o32_max + 4.0 * float(fp32_ulp(torch.tensor([gmax]))[0])
        record(f"{name} grad[{k}] gpu vs fp64", st_gpu, floor=floor, bound_abs=bound)
        record(f"{name} grad[{k}] oracle32 vs fp64", st_o32, floor=floor)
        assert st_gpu["max_abs"] <= bound, (name, k, st_gpu["max_abs"], o32_max)
        worst_ratio_t = max(worst_ratio_t, st_gpu["max_abs"] / max(o32_max, 1e-30))
        # per element: the pre-round-3 bound (1e-4 of the element's magnitude + 2e-6 of the
        # tensor's largest) plus 4x the fp32 oracle's own distance to float64 on that element
        # (largest over the four fp32 evaluations): where the TD error cancels most of Q the fp32
        # oracle itself exceeds the pre-round-3 bound (up to 3.6x at C5's first fused tick)
        noise = torch.stack([(c - b).abs() for c in cs]).max(dim=0).values
        old = 1e-4 * b.abs() + floor
        elem_bound = old + 4.0 * noise
        ratio = float(((a - b).abs() / elem_bound).max())
        record(f"{name} grad[{k}] elementwise: largest error / bound", {
            "gpu": ratio, "gpu_over_pre_r3_bound": float(((a - b).abs() / old).max()),
            "oracle32_over_pre_r3_bound": float(((cs[0] - b).abs() / old).max())})
        if ratio > worst_elem:
            worst_elem, worst_k = ratio, k
        o += n
    record(f"{name} grad: worst per-tensor ratio gpu/oracle32 error", {"ratio": worst_ratio_t,
                                                                       "worst_elementwise_ratio": worst_elem})
    assert worst_elem <= 1.0, (f"{name}: a {worst_k} gradient element outside 1e-4 rel + 2e-6 x tensor max + "
                               f"4x the fp32 oracle's own error on it (ratio {worst_elem:.3f})")


def _adam_check(name, p_gpu, m_gpu, v_gpu, p0, g_gpu, m0, v0, step0, norm_gpu=None, lr=1e-3, b1=0.9, b2=0.999):
    """clip_grad_norm_ + Adam of the GPU, isolated from the gradient: against torch on the GPU's
    OWN gradient (module docstring for the bounds)."""
    m0 = torch.zeros_like(p0) if m0 is None else m0
    v0 = torch.zeros_like(p0) if v0 is None else v0
    ref_p, ref_m, ref_v, ref_norm = O.clip_adam(p0, g_gpu, m0, v0, step0)
    if norm_gpu is not None:
        st = error_stats(torch.tensor([norm_gpu]), torch.tensor([ref_norm]))
        record(f"{name} clip total_norm (own gradient)", st)
        assert st["max_ulp"] <= 8, st
    coef = min(1.0, 1.0 / (ref_norm + 1e-6))
    gc = g_gpu.double() * coef
    m_terms = b1 * m0.double().abs() + (1 - b1) * gc.abs()
    v_terms = b2 * v0.double().abs() + (1 - b2) * gc * gc
    st_m = error_stats(m_gpu, ref_m, scale=m_terms)
    st_v = error_stats(v_gpu, ref_v, scale=v_terms)
    st_p = error_stats(p_gpu, ref_p, scale=torch.full_like(p_gpu, lr, dtype=torch.float64))
    record(f"{name} adam m (own gradient)", st_m, tol_ulp=8)
    record(f"{name} adam v (own gradient)", st_v, tol_ulp=16)
    record(f"{name} weights after Adam (own gradient)", st_p, tol_ulp=4)
    assert st_m["max_ulp"] <= 8, st_m
    assert st_v["max_ulp"] <= 16, st_v
    assert st_p["max_ulp"] <= 4, st_p


def _compare_update(name, eng, p0, t0, idx, S, N, scen, conv):
    s, a, r, s1 = _rows(eng, idx, scen, name)
    loss32, g32s, loss64, g64 = oracle_grad_orders(p0, t0, s, a, r, s1, conv=conv, seed=S + N)
    grad = eng.grad.cpu()
    loss = grad[O.N_PARAMS].double().item() / (S * N)
    # TD loss: north_star 1e-5 vs the fp32 oracle, and in ulps vs fp64: within 4x the fp32
    # oracle's own error + 8 ulps (observed round 3: <= 34 ulps, the oracle's own <= 38)
    assert_close_rel(loss, loss32, 1e-5, f"{name} TD loss vs oracle32")
    st_gpu = error_stats(torch.tensor([loss]), torch.tensor([loss64]))
    st_o32 = error_stats(torch.tensor([loss32]), torch.tensor([loss64]))
    record(f"{name} TD loss gpu vs fp64", st_gpu)
    record(f"{name} TD loss oracle32 vs fp64", st_o32)
    assert st_gpu["max_ulp"] <= 4.0 * st_o32["max_ulp"] + 8.0, (st_gpu, st_o32)
    _record_forward_rounding(name, grad[:O.N_PARAMS], g32s[:-1], g32s[-1], g64)
    _grad_bound_check(name, grad[:O.N_PARAMS], g32s, g64)
    return g32s[0], grad[:O.N_PARAMS].clone()


def _record_forward_rounding(name, g_gpu, g32s, g_cr, g64):
    """Recorded (round 6): the correctly-rounded-linear evaluation g_cr and the GPU, each as a
    multiple of the spread of the other four fp32 evaluations g32s, which was the bound's spread
    until round 6.  Three of those four share torch's per-node rounding of Q, which the TD error
    amplifies, so that spread under-states what a different fp32 forward legitimately moves: g_cr
    reached 10.5x of it (C3 GCN), where a 4x bound on it would reject a MORE accurate evaluation.
    tools/fwd_rounding.py, profiles/r06_fwd_rounding.json."""
    o, worst_cr, worst_gpu, worst_both = 0, (0.0, None), (0.0, None), 0.0
    for k, shape in O.PARAM_ORDER:
        n = 1
        for d in shape:
            n *= d
        b = g64[o:o + n]
        spread = max(float((g[o:o + n].double() - b).abs().max()) for g in g32s)
        if spread > 0.0:
            e_cr = float((g_cr[o:o + n].double() - b).abs().max())
            e_gpu = float((g_gpu[o:o + n].double() - b).abs().max())
            worst_cr = max(worst_cr, (e_cr / spread, k), key=lambda x: x[0])
            worst_gpu = max(worst_gpu, (e_gpu / spread, k), key=lambda x: x[0])
            worst_both = max(worst_both, e_gpu / max(spread, e_cr))
        o += n
    record(f"{name} grad: correctly-rounded-linear fp32 evaluation vs the four-evaluation spread", {
        "cr_ratio": worst_cr[0], "cr_tensor": worst_cr[1], "gpu_ratio": worst_gpu[0], "gpu_tensor": worst_gpu[1],
        "gpu_over_five_evaluation_spread": worst_both})


def _clip_adam64(p0, g, m0, v0, step0, lr=1e-3, b1=0.9, b2=0.999, eps=1e-8, max_norm=1.0):
    """clip_grad_norm_ + one torch.optim.Adam step (train_gcn_dqn.py:85,125-126), in float64."""
    p0, g = p0.double(), g.double()
    m0 = torch.zeros_like(p0) if m0 is None else m0.double()
    v0 = torch.zeros_like(p0) if v0 is None else v0.double()
    coef = min(1.0, max_norm / (float(g.norm()) + 1e-6))
    gc = g * coef
    m, v, t = b1 * m0 + (1 - b1) * gc, b2 * v0 + (1 - b2) * gc * gc, step0 + 1
    return p0 - (lr / (1 - b1 ** t)) * m / ((v / (1 - b2 ** t)).sqrt() + eps)


def _end_to_end_weights(name, p_gpu, p0, g32, m0, v0, step0, g_gpu=None):
    """weights after Adam vs torch's update on the fp32 oracle's gradient: within 2e-6, plus, per
    element, the difference that Adam itself makes of the two gradients' difference (both updates in
    float64).  Adam normalises each element by sqrt(v) + eps, so where a clipped gradient element is
    near eps = 1e-8 the update moves by up to lr * |dg| / (4 eps): the first C5 N = 6 fused tick has
    such an element, where the two fp32 gradients' last-bit difference (both within the gradient
    bounds of _grad_bound_check) became 1.1e-5 of weight.  Adam's own arithmetic is checked apart
    from the gradient, in ulps, by _adam_check."""
    ref_p, _, _, ref_norm = O.clip_adam(p0, g32, torch.zeros_like(p0) if m0 is None else m0,
                                        torch.zeros_like(p0) if v0 is None else v0, step0)
    st = error_stats(p_gpu, ref_p)
    allow = torch.full_like(p_gpu, 2e-6, dtype=torch.float64)
    if g_gpu is not None:
        sens = (_clip_adam64(p0, g_gpu, m0, v0, step0) - _clip_adam64(p0, g32, m0, v0, step0)).abs()
        allow = allow + sens
        st["elements_over_2e-6_explained_by_the_gradient_difference"] = int(
            ((p_gpu.double() - ref_p.double()).abs() > 2e-6).sum())
    ratio = float(((p_gpu.double() - ref_p.double()).abs() / allow).max())
    st["largest_error_over_allowance"] = ratio
    record(f"{name} weights after Adam vs the oracle-gradient update", st)
    assert ratio <= 1.0, st
    return ref_norm


@pytest.mark.parametrize("name,scen,N,B,S,conv", CASES)
def test_td_api_update_at_benchmark_size(sw, golden_weights, name, scen, N, B, S, conv):
    """swarm_td_grad + swarm_grad_reduce + swarm_adam_step (the reference-shaped
    train_step_dqn) on S graphs drawn from a 4-slot ring of real transitions."""
    slots = 4
    p = _weights(golden_weights, scen, 5)
    tgt = _weights(golden_weights, scen, 6)
    eng = sw.SwarmEngine(scen, N, B, seed=12, params=p, batch=S, replay_capacity=slots * B, eps=0.3,
                         update_target_every=100000, conv=conv)
    _prefill(eng, slots)
    eng.target.copy_(tgt.cuda())
    idx = torch.randperm(slots * B, generator=torch.Generator().manual_seed(S + N))[:S].to(torch.int32)
    p0, t0 = eng.params.cpu().clone(), eng.target.cpu().clone()
    eng.td_grad(sample_in=idx.cuda())
    torch.cuda.synchronize()
    g32, g_gpu = _compare_update(name, eng, p0, t0, idx, S, N, scen, conv)
    eng.adam()
    torch.cuda.synchronize()
    c = eng.read_ctrl()
    assert c["adam_step"] == 1
    ref_norm = _end_to_end_weights(name, eng.params.cpu(), p0, g32, None, None, 0, g_gpu=g_gpu)
    assert ref_norm > 1.0, "the clip must be active at these sizes (norm > max_norm)"
    assert_close_rel(c["grad_norm"], ref_norm, 1e-5, f"{name} clip total_norm")
    _adam_check(name, eng.params.cpu(), eng.adam_m.cpu(), eng.adam_v.cpu(), p0, g_gpu, None, None, 0,
                norm_gpu=c["grad_norm"])


@pytest.mark.parametrize("name,scen,N,B,S,conv", CASES)
def test_fused_tick_update_at_benchmark_size(sw, golden_weights, name, scen, N, B, S, conv):
    """The headline launch (swarm_train_tick + swarm_reduce_advance) at its benchmarked size:
    two consecutive training ticks.  The first tick's gradient (from the initial weights) and
    the second's (after the first's deferred clip + Adam, applied in the second launch's
    prologue) against the oracle on the batch each tick drew, including the graphs drawn from
    the tick's own slot (hand-off records)."""
    slots = 3
    p = _weights(golden_weights, scen, 5)
    eng = sw.SwarmEngine(scen, N, B, seed=13, params=p, batch=S, replay_capacity=(slots + 2) * B, eps=0.3,
                         update_target_every=100000, conv=conv)
    assert eng.fused
    _prefill(eng, slots)
    target = eng.target.cpu().clone()
    prev = None   # (weights, fp32-oracle gradient, GPU gradient, m, v, step) of the previous tick
    for t in range(2):
        ws = eng.read_ctrl()["write_slot"]
        eng.train_tick(full_out=False)
        torch.cuda.synchronize()
        assert eng.handoff_errors() == 0
        # the weights this tick used: its prologue applied the previous tick's pending step and
        # the reduce copied them to the current rows
        p_used, m_used, v_used = eng.params.cpu().clone(), eng.adam_m.cpu().clone(), eng.adam_v.cpu().clone()
        if prev is not None:
            pw, g32p, ggp, mp, vp, sp = prev
            _end_to_end_weights(f"{name} fused tick {t}", p_used, pw, g32p, mp, vp, sp, g_gpu=ggp)
            _adam_check(f"{name} fused tick {t}", p_used, m_used, v_used, pw, ggp, mp, vp, sp)
        idx = eng.samples.cpu().clone()
        assert len(set(idx.tolist())) == S
        n_cur = int(((idx.long() // B) == ws).sum())
        assert n_cur > 0, "some graphs come from the tick's own slot"
        record(f"{name} fused tick {t}: graphs from the tick's own slot", {"n": n_cur})
        g32, g_gpu = _compare_update(f"{name} fused tick {t}", eng, p_used, target, idx, S, N, scen, conv)
        prev = (p_used, g32, g_gpu, m_used, v_used, t)
    eng.flush()
    torch.cuda.synchronize()
    pw, g32p, ggp, mp, vp, sp = prev
    _end_to_end_weights(f"{name} fused flushed second step", eng.params.cpu(), pw, g32p, mp, vp, sp, g_gpu=ggp)
    _adam_check(f"{name} fused flushed second step", eng.params.cpu(), eng.adam_m.cpu(), eng.adam_v.cpu(), pw, ggp,
                mp, vp, sp)


def test_fused_tick_target_sync_at_benchmark_size(sw, golden_weights):
    """VERDICT r4 "next" #5: the fused tick's target sync (train_gcn_dqn.py:131-133: after the
    optimizer step of reference tick `ticks`, target <- model when ticks % update_target_every == 0)
    at C2's size with update_target_every = 2.  The update of tick t is applied in tick t + 1's
    prologue, which also writes the target row when (t + 1) % every == 0, and that tick's TD blocks
    already use the synced target.  Checked against the oracle: the synced target equals the
    post-step weights bit for bit and torch's update on the fp32 oracle's gradient within 2e-6; the
    next tick's gradient (computed against the synced target) passes the oracle bounds; the tick
    after it leaves the target alone."""
    name, scen, N, B, S, conv = "C2 sync", "GoTo", 8, 1024, 1024, "gat"
    p = _weights(golden_weights, scen, 5)
    eng = sw.SwarmEngine(scen, N, B, seed=14, params=p, batch=S, replay_capacity=6 * B, eps=0.3,
                         update_target_every=2, conv=conv)
    assert eng.fused
    _prefill(eng, 3)
    assert eng.read_ctrl()["tick"] == 3
    t0 = eng.target.cpu().clone()
    # tick 3: nothing pending yet (prefill does not train), its TD uses the initial target
    eng.train_tick()
    torch.cuda.synchronize()
    p3 = eng.params.cpu().clone()
    g32, g_gpu = _compare_update(f"{name} tick 3", eng, p3, t0, eng.samples.cpu().clone(), S, N, scen, conv)
    assert torch.equal(eng.target.cpu(), t0)
    # tick 4: its prologue applies tick 3's step and syncs (4 % 2 == 0)
    eng.train_tick()
    torch.cuda.synchronize()
    assert eng.handoff_errors() == 0
    w4, tgt4 = eng.params.cpu().clone(), eng.target.cpu().clone()
    assert not torch.equal(w4, p3) and torch.equal(tgt4, w4), "the target row is the post-step weights"
    _end_to_end_weights(f"{name} synced target", tgt4, p3, g32, None, None, 0, g_gpu=g_gpu)
    _adam_check(f"{name} synced target", tgt4, eng.adam_m.cpu(), eng.adam_v.cpu(), p3, g_gpu, None, None, 0)
    _compare_update(f"{name} tick 4 (synced target)", eng, w4, tgt4, eng.samples.cpu().clone(), S, N, scen, conv)
    # tick 5: step applied, no sync (5 % 2 != 0)
    eng.train_tick()
    torch.cuda.synchronize()
    assert not torch.equal(eng.params.cpu(), w4) and torch.equal(eng.target.cpu(), tgt4)
