"""CPU-only tests: library exports, neighbour-set semantics, oracle self-consistency,
host-side API objects.  No GPU compute is called here."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from oracle import knn_select, philox
from oracle import swarm_oracle as O
from tests.conftest import assert_close_rel

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _host_lib():
    import swarm_amd._lib as L
    if not os.path.exists(L.LIB_PATH):
        import __graft_entry__
        __graft_entry__.build()
    return L, L.load(require_gpu=False)


def test_library_exports_every_header_symbol():
    L, lib = _host_lib()
    hdr = open(os.path.join(ROOT, "include", "swarm_hip.h")).read()
    names = set(re.findall(r"^\s*(?:int|int64_t|uint32_t|const char\*)\s+(swarm_\w+)\(", hdr, re.M))
    assert len(names) >= 15
    raw = ctypes.CDLL(L.LIB_PATH)
    for n in sorted(names):
        assert hasattr(raw, n), n
    assert names == set(L.EXPORTED)
    assert lib.swarm_abi_version() == L.ABI_VERSION == 10 and lib.swarm_n_params() == O.N_PARAMS


def test_integration_guide_names_every_entry_point():
    """INTEGRATION.md §3 says where each C entry point plugs into the reference: every symbol
    include/swarm_hip.h declares appears there."""
    hdr = open(os.path.join(ROOT, "include", "swarm_hip.h")).read()
    names = set(re.findall(r"^\s*(?:int|int64_t|uint32_t|const char\*)\s+(swarm_\w+)\(", hdr, re.M))
    guide = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    assert sorted(n for n in names if f"`{n}" not in guide and f"{n}`" not in guide) == []


def test_topk_emulation_matches_torch_fixture():
    z = np.load(os.path.join(ROOT, "tests", "golden", "topk_ties.npz"))
    for row, (n, k), s in zip(z["dist"], z["nk"], z["sets"]):
        assert knn_select.topk_smallest_set(row[:n], int(k)) == sorted(np.where(s)[0].tolist())


def test_lane_parallel_topk_restatement_matches_torch():
    """The lane-parallel partition step of the device's tie path (csrc/swarm_dl.h
    knn_tie_rows_wave, restated as knn_select.nth_element_lanes) selects torch.topk's set: the
    committed tie fixture, 3,000 fresh tie-heavy rows against torch.topk itself, and a row that
    ends in heap_select (depth limit)."""
    import random
    import torch
    z = np.load(os.path.join(ROOT, "tests", "golden", "topk_ties.npz"))
    for row, (n, k), s in zip(z["dist"], z["nk"], z["sets"]):
        assert knn_select.topk_smallest_set_lanes(row[:n], int(k)) == sorted(np.where(s)[0].tolist())
    rng = random.Random(7)
    for trial in range(3000):
        n = rng.randint(4, 16)
        k = rng.randint(1, n)
        if trial % 2:
            vals = [float(rng.randint(0, 3)) for _ in range(n)]
        else:
            vals = [rng.choice([0.15, 0.3, 0.2121, 0.3354]) for _ in range(n)]
        d = torch.tensor(vals, dtype=torch.float32)
        want = sorted(torch.topk(d, k, largest=False).indices.tolist())
        assert knn_select.topk_smallest_set_lanes(d.tolist(), k) == want, (vals, k)
    vals, k = knn_select.HEAP_PATH_ROW
    d = torch.tensor(vals, dtype=torch.float32)
    want = sorted(torch.topk(d, k, largest=False).indices.tolist())
    assert knn_select.topk_smallest_set_lanes(vals, k) == knn_select.topk_smallest_set(vals, k) == want


def test_slot_exchange_topk_restatement_matches_torch():
    """Round 3's straight-line tie path (partners through rank slots, the finish as a stable-rank
    set; knn_select.topk_smallest_set_slots) selects torch.topk's set on the committed fixture,
    3,000 fresh tie-heavy rows and the heap_select row."""
    import random
    z = np.load(os.path.join(ROOT, "tests", "golden", "topk_ties.npz"))
    for row, (n, k), s in zip(z["dist"], z["nk"], z["sets"]):
        assert knn_select.topk_smallest_set_slots(row[:n], int(k)) == sorted(np.where(s)[0].tolist())
    rng = random.Random(13)
    for trial in range(3000):
        n = rng.randint(4, 16)
        k = rng.randint(1, n)
        vals = ([float(rng.randint(0, 3)) for _ in range(n)] if trial % 2 else
                [rng.choice([0.15, 0.3, 0.2121, 0.3354]) for _ in range(n)])
        d = torch.tensor(vals, dtype=torch.float32)
        want = sorted(torch.topk(d, k, largest=False).indices.tolist())
        assert knn_select.topk_smallest_set_slots(d.tolist(), k) == want, (vals, k)
    vals, k = knn_select.HEAP_PATH_ROW
    assert knn_select.topk_smallest_set_slots(vals, k) == knn_select.topk_smallest_set(vals, k)


def test_rank_signature_fixes_the_topk_set():
    """The acting rollout's tie memo (csrc/swarm_dl.h knn_masks_wave) reuses a slot's last tie
    result when the row's rank signature lt_j = #{l : d_l < d_j} repeats.  Pinned against the
    reference's own call, torch.topk: rows mapped through random strictly increasing value maps
    keep their signature and their set, and across 20,000 random tie-heavy rows every signature
    has one set."""
    import random
    rng = random.Random(17)
    seen = {}
    for trial in range(20000):
        n = rng.randint(4, 10)
        k = rng.randint(1, n - 1)
        vals = [float(rng.randint(0, 4)) for _ in range(n)]
        d = torch.tensor(vals, dtype=torch.float32)
        want = sorted(torch.topk(d, k, largest=False).indices.tolist())
        sig = knn_select.rank_signature(vals)
        key = (n, k, sig)
        assert seen.setdefault(key, want) == want, (vals, k)
        if trial % 10 == 0:   # a strictly increasing map of the distinct values
            levels = sorted(set(vals))
            new = sorted(rng.uniform(0.0, 2.0) for _ in levels)
            if len(set(new)) == len(new):
                f = dict(zip(levels, new))
                mapped = [f[v] for v in vals]
                assert knn_select.rank_signature(mapped) == sig
                dm = torch.tensor(mapped, dtype=torch.float32)
                assert sorted(torch.topk(dm, k, largest=False).indices.tolist()) == want, (vals, mapped, k)
    assert len(seen) > 1000


def test_host_topk_matches_torch_fixture():
    """The C++ selection the kernels run (swarm_knn.h), compiled for the host."""
    L, lib = _host_lib()
    z = np.load(os.path.join(ROOT, "tests", "golden", "topk_ties.npz"))
    sel = (ctypes.c_uint8 * 32)()
    for row, (n, k), s in zip(z["dist"], z["nk"], z["sets"]):
        d = np.ascontiguousarray(row[:n], dtype=np.float32)
        rc = lib.swarm_host_topk_set(d.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), int(n), int(k), sel)
        assert rc == 0
        assert [j for j in range(n) if sel[j]] == sorted(np.where(s)[0].tolist())
    assert lib.swarm_host_topk_set(np.zeros(4, np.float32).ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                   4, 5, sel) == -2


def test_host_topk_random_ties_vs_torch():
    L, lib = _host_lib()
    rng = np.random.default_rng(7)
    sel = (ctypes.c_uint8 * 32)()
    for _ in range(2000):
        n = int(rng.integers(1, 33))
        k = int(rng.integers(1, n + 1))
        d = (rng.integers(0, 5, size=n).astype(np.float32) * np.float32(0.1)).astype(np.float32)
        _, idx = torch.topk(torch.tensor(d), k, largest=False)
        lib.swarm_host_topk_set(d.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), n, k, sel)
        assert [j for j in range(n) if sel[j]] == sorted(idx.tolist())


def test_philox_known_answers():
    kat = [((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
           ((0xffffffff,) * 4, (0xffffffff, 0xffffffff), (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
           ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
            (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1))]
    for c, k, e in kat:
        assert tuple(int(x) for x in philox.philox4x32(*c, *k)) == e


def test_sample_index_is_a_permutation():
    for n in (1, 2, 3, 7, 64, 100, 1000):
        got = sorted(O.sample_index(i, n, seed=5, rnd=3) for i in range(n))
        assert got == list(range(n))


def test_host_sample_permutation_and_inverse_match_oracle():
    """The keyed batch permutation the kernels draw (swarm_common.h sample_index) matches the
    oracle's restatement, and sample_position — which the fused tick's acting waves use to
    decide whether their env's transition is in this tick's TD batch — is its inverse."""
    L, lib = _host_lib()
    for n, seed, rnd in ((1, 0, 0), (7, 5, 3), (1024, 0, 101), (1000, 3, 7), (8192 * 3 + 5, 11, 200)):
        k0, k1 = (int(x) for x in philox.seed_key(seed))
        idx = [lib.swarm_host_sample_index(i, n, k0, k1, rnd) for i in range(min(n, 300))]
        assert idx == [O.sample_index(i, n, seed=seed, rnd=rnd) for i in range(min(n, 300))]
        assert [lib.swarm_host_sample_position(g, n, k0, k1, rnd) for g in idx] == list(range(len(idx)))
        if n <= 1024:
            assert sorted(lib.swarm_host_sample_position(g, n, k0, k1, rnd) for g in range(n)) == list(range(n))


def test_fused_tick_support_and_workspace_host_side():
    """swarm_train_tick's host-side contract (no GPU call): which configurations have a
    one-launch tick, its workspace size (512 B: the error word, and the opt-in one-launch tick's
    epoch and two counters, one 128-B line each; then one 128-B-aligned granule record per env),
    and the error codes it returns before launching anything."""
    L, lib = _host_lib()
    def cfg(B=1024, N=8, graph=0, k=5, conv=0, radius=0.0, scen=0):
        return L.SwarmConfig(B, N, scen, graph, k, conv, 0, 0, 0, radius, 0)
    ok = [cfg(), cfg(N=16), cfg(N=12, conv=1), cfg(graph=1, k=5), cfg(graph=3, radius=0.3), cfg(B=1, N=1),
          cfg(scen=1), cfg(scen=2, N=2), cfg(scen=2, N=12, graph=1, k=5)]
    bad = [cfg(N=17), cfg(N=32), cfg(graph=2), cfg(graph=1, k=9), cfg(graph=3, radius=0.0), cfg(B=0),
           cfg(scen=2, N=1), cfg(scen=3)]
    for c in ok:
        assert lib.swarm_train_tick_supported(ctypes.byref(c)) == 1
        n_gran = -(-10 * c.n_agents // 16) * 16
        assert lib.swarm_train_tick_workspace_bytes(ctypes.byref(c)) == 512 + c.n_envs * n_gran * 8
    for c in bad:
        assert lib.swarm_train_tick_supported(ctypes.byref(c)) == 0
        assert lib.swarm_train_tick_workspace_bytes(ctypes.byref(c)) == -4
    hp = L.SwarmAdamCfg(1e-3, 0.9, 0.999, 1e-8, 1.0, 0.99, 32, 200, 1, 0)
    lr = L.SwarmLearner(*([1] * 8))
    rp = L.SwarmReplay(1, 1, 1, 1, 4, 0)
    args = (ctypes.byref(hp), ctypes.byref(lr), 1, ctypes.byref(rp), 1, None, 1, 1, None, None)
    assert lib.swarm_train_tick(ctypes.byref(bad[0]), *args) == -4
    assert lib.swarm_train_tick(ctypes.byref(ok[0]), *args[:6], 1, None, None, None) == -1   # no workspace
    # the three-layer GAT (Flocking checkpoints) is forward only: every learner entry point refuses it
    g3 = L.SwarmConfig(64, 8, 2, 0, 5, 0, 0, 0, 0, 0.0, L.NET_GAT3)
    assert lib.swarm_train_tick_supported(ctypes.byref(g3)) == 0
    assert lib.swarm_td_grad(ctypes.byref(g3), ctypes.byref(hp), 1, 1, ctypes.byref(rp), 1, None, None, 1,
                             None) == -4
    assert lib.swarm_train_act_step(ctypes.byref(g3), ctypes.byref(hp), ctypes.byref(lr), 1, ctypes.byref(rp), 1,
                                    None, None, None) == -4


@pytest.mark.parametrize("n", [1, 5, 8, 12])
def test_dense_forward_equals_edge_list_forward(golden_weights, n):
    params = O.unflatten_params(torch.tensor(golden_weights["go_to"][1]))
    g = torch.Generator().manual_seed(n)
    B = 6
    pos = torch.randn(B, n, 2, generator=g) * 0.3
    vel = torch.randn(B, n, 2, generator=g) * 0.1
    x = O.node_features(pos, vel)
    for mult in (O.multiplicity_complete(B, n), O.multiplicity_knn(O.knn_sets(pos, min(3, n))),
                 O.multiplicity_radius(O.radius_sets(pos, 0.3))):
        qd = O.q_forward_dense(params, x, mult)
        qe = O.q_forward_edges(params, x.reshape(B * n, 7), O.edge_index_from_multiplicity(mult))
        assert_close_rel(qd.reshape(B * n, 9), qe, 1e-5, 'dense vs edge-list Q')


def test_edge_builders_match_multiplicity():
    pos = torch.tensor(O.grid_offsets(9), dtype=torch.float32)
    ei = O.knn_edge_index(pos, 5)
    m = O.multiplicity_knn(O.knn_sets(pos[None], 5))[0]
    cnt = torch.zeros(9, 9)
    for s, d in ei.t().tolist():
        cnt[s, d] += 1
    assert torch.equal(cnt, m)
    ec = O.complete_edge_index(6)
    cnt = torch.zeros(6, 6)
    for s, d in ec.t().tolist():
        cnt[s, d] += 1
    assert torch.equal(cnt, O.multiplicity_complete(1, 6)[0])


def test_radius_builders_match_multiplicity():
    """Radius-neighbour graph (north_star; not in the reference): symmetric sets without
    self-pairs, the edge list and the multiplicity agree, and (0, 0) is appended."""
    pos = torch.tensor(O.grid_offsets(9), dtype=torch.float32)
    for r in (0.1, 0.15, 0.22, 1.0):
        sets = O.radius_sets(pos[None], r)[0]
        assert torch.equal(sets, sets.t()) and not sets.diagonal().any()
        ei = O.radius_edge_index(pos, r)
        cnt = torch.zeros(9, 9)
        for s_, d_ in ei.t().tolist():
            cnt[s_, d_] += 1
        assert torch.equal(cnt, O.multiplicity_radius(sets[None])[0])
    assert int(O.radius_sets(pos[None], 1.0)[0].sum()) == 9 * 8


def test_radius_graph_host_builder():
    import swarm_amd
    obs = {f"agent{i}": torch.randn(3, 6) for i in range(4)}
    d = swarm_amd.create_radius_graph_from_observations(obs, 4, 0.5)
    assert d.swarm["graph"] == 3 and d.swarm["radius"] == 0.5 and d.x.shape == (12, 7)
    with pytest.raises(ValueError):
        swarm_amd.create_radius_graph_from_observations(obs, 4, 0.0)


def test_td_step_oracle_reduces_loss(golden_weights):
    """Sanity of the oracle learner itself: repeated updates on one batch lower the loss."""
    p = torch.tensor(golden_weights["go_to"][2])
    g = torch.Generator().manual_seed(0)
    S, N = 4, 5
    s = torch.randn(S, N, 4, generator=g) * 0.5
    s1 = torch.randn(S, N, 4, generator=g) * 0.5
    a = torch.randint(0, 9, (S, N), generator=g)
    r = torch.randn(S, N, generator=g)
    m = torch.zeros_like(p)
    v = torch.zeros_like(p)
    losses = []
    tgt = p.clone()
    for step in range(30):
        out = O.td_step(p, tgt, m, v, step, s, a, r, s1)
        p, m, v = out["params"], out["m"], out["v"]
        losses.append(out["loss"])
    assert losses[-1] < losses[0]


@pytest.mark.parametrize("conv", ["gat", "gcn"])
def test_correctly_rounded_linears_evaluation(golden_weights, conv):
    """The fifth fp32 evaluation the large parity tests record (oracle.correctly_rounded_linears):
    every Q of it is within one fp32 ulp of the float64 evaluation's (observed <= 0.78 ulp; torch's fp32
    Q up to 3.7 ulp), its gradient is fp32, and leaving the context restores torch's F.linear."""
    p = torch.tensor(golden_weights["obstacle_avoidance"][5])
    t = torch.tensor(golden_weights["obstacle_avoidance"][6])
    g = torch.Generator().manual_seed(1)
    S, N = 16, 7
    s = torch.cat([torch.rand(S, N, 2, generator=g) * 2 - 1, torch.randn(S, N, 2, generator=g) * 0.1], -1)
    s1 = s + torch.randn(S, N, 4, generator=g) * 0.01
    a = torch.randint(0, 9, (S, N), generator=g)
    r = torch.randn(S, N, generator=g)
    lin0 = torch.nn.functional.linear
    _, g32, q32, _ = O.td_loss_grad(p, t, s, a, r, s1, conv=conv)
    with O.correctly_rounded_linears():
        assert torch.nn.functional.linear is not lin0
        _, gcr, qcr, _ = O.td_loss_grad(p, t, s, a, r, s1, conv=conv)
    assert torch.nn.functional.linear is lin0
    _, _, q64, _ = O.td_loss_grad(p, t, s, a, r, s1, conv=conv, dtype=torch.float64)
    assert gcr.dtype == torch.float32 and qcr.dtype == torch.float32
    ulp = torch.from_numpy(np.spacing(np.abs(q64.numpy()).astype(np.float32)).astype(np.float64))
    e_cr, e_32 = (qcr.double() - q64).abs() / ulp, (q32.double() - q64).abs() / ulp
    assert float(e_cr.max()) <= 1.0 and float(e_cr.mean()) < float(e_32.mean())
    assert torch.allclose(gcr, g32, rtol=1e-3, atol=1e-5)


def test_gcn_module_state_dict_matches_reference_layout(golden_weights):
    import swarm_amd
    model = swarm_amd.GCN(7, 32, 9)
    keys = list(model.state_dict().keys())
    assert keys == [k for k, _ in O.PARAM_ORDER]
    sd = O.unflatten_params(torch.tensor(golden_weights["obstacle_avoidance"][3]))
    model.load_state_dict(sd)
    assert torch.equal(model.flat_params("cpu"), torch.tensor(golden_weights["obstacle_avoidance"][3]))


def test_graph_builders_host_side():
    import swarm_amd
    obs = {f"agent{i}": torch.randn(3, 6) for i in range(5)}
    d = swarm_amd.create_graph_from_observations(obs)
    assert d.x.shape == (15, 7) and d.swarm["n_graphs"] == 3
    assert torch.equal(d.x.view(3, 5, 7)[..., 6], torch.arange(5.0).expand(3, 5))
    with pytest.raises(RuntimeError):
        swarm_amd.create_knn_graph_from_observations(obs, 5, k=10)
    b = swarm_amd.Batch.from_data_list([d, d])
    assert b.swarm["n_graphs"] == 6 and b.x.shape == (30, 7)


def test_engine_refuses_cpu():
    import swarm_amd
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError):
        swarm_amd.SwarmEngine("GoTo", 8, 4)


def test_library_is_current_by_source_digest(tmp_path):
    """build._current: a library whose file time is older than the sources (a checkout touched
    them) still counts as current when it carries the digest of the sources as they are now;
    another digest does not."""
    from swarm_amd import build as b
    old = min(os.path.getmtime(f) for f in b._deps()) - 100.0
    good, bad = tmp_path / "good.so", tmp_path / "bad.so"
    good.write_bytes(b"\x7fELF...libswarm_hip gfx950 abi 9 src " + b.source_digest().encode() + b"\x00")
    bad.write_bytes(b"\x7fELF...libswarm_hip gfx950 abi 9 src 0123456789abcdef\x00")
    for f in (good, bad):
        os.utime(f, (old, old))
    assert b._current(str(good)) and not b._current(str(bad))
    assert not b._current(str(tmp_path / "missing.so"))
    # a variant's digest covers its extra flags
    assert not b._current(str(good), ["-DSWARM_STAMPS=2"])
