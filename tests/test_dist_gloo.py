"""Multi-rank contract of the training tick on CPU (gloo, world size 2).

SURVEY.md §8(e): envs shard contiguously by global index, each rank samples its
own replay, ONE sum all-reduce of the flat gradient, then clip + Adam on grad / W
identically on every rank == the single-process update over the union batch.
The per-rank gradient is the oracle's (tests' checker); the sharding and the
collective are the product's host code (swarm_amd.dist).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import swarm_amd.dist as swdist
from oracle import swarm_oracle as O

WORLD = 2
S_PER_RANK, N = 3, 5


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _global_batch(seed=0):
    """Synthetic replay batch of WORLD * S_PER_RANK graphs (global graph order = rank-major)."""
    g = torch.Generator().manual_seed(seed)
    S = WORLD * S_PER_RANK
    s = torch.randn(S, N, 4, generator=g) * 0.3
    s1 = s + torch.randn(S, N, 4, generator=g) * 0.05
    a = torch.randint(0, 9, (S, N), generator=g)
    r = -torch.rand(S, N, generator=g) * 3
    w = O.flatten_params({k: torch.randn(shape, generator=g) * 0.3 for k, shape in O.PARAM_ORDER})
    tw = w + torch.randn(w.shape, generator=g) * 0.01
    m = torch.randn(O.N_PARAMS, generator=g) * 1e-3
    v = torch.rand(O.N_PARAMS, generator=g) * 1e-4
    return s, a, r, s1, w, tw, m, v


def _rank_main(rank, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD))
    torch.set_num_threads(1)
    pg = swdist.init_process_group("gloo")
    shard = swdist.Shard(rank, WORLD, S_PER_RANK)
    s, a, r, s1, w, tw, m, v = _global_batch()
    sl = slice(shard.env_offset, shard.env_offset + S_PER_RANK)
    loss, grad, _, _ = O.td_loss_grad(w, tw, s[sl], a[sl], r[sl], s1[sl])
    buf = torch.cat([grad, torch.tensor([loss])])         # flat gradient + loss, as the engine's grad buffer
    swdist.allreduce_grad_(buf, WORLD, pg)
    buf = buf / WORLD                                      # swarm_adam_cfg.world_size scaling
    newp, nm, nv, norm = O.clip_adam(w, buf[:O.N_PARAMS], m, v, adam_step=3)
    torch.save(dict(params=newp, m=nm, v=nv, norm=norm, loss=float(buf[-1])), f"{out_path}.{rank}")
    dist.barrier()
    dist.destroy_process_group()


def test_shard_ranges():
    shards = [swdist.Shard(r, 4, 1024) for r in range(4)]
    assert [sh.env_offset for sh in shards] == [0, 1024, 2048, 3072]
    assert shards[0].global_envs == 4096
    covered = sorted(e for sh in shards for e in sh.env_range())
    assert covered == list(range(4096))


def test_reset_is_layout_independent():
    """Per-rank resets keyed by env_offset concatenate to the single-rank reset."""
    full = O.reset_centres(O.SCENARIO_GOTO, 8, seed=3, episode=5, shared=False)
    parts = [O.reset_centres(O.SCENARIO_GOTO, 4, seed=3, episode=5, shared=False, env_offset=sh.env_offset)
             for sh in (swdist.Shard(0, 2, 4), swdist.Shard(1, 2, 4))]
    assert torch.equal(torch.cat(parts), full)


def test_allreduce_equals_union_batch(tmp_path):
    out = str(tmp_path / "rank")
    mp.start_processes(_rank_main, args=(_free_port(), out), nprocs=WORLD, join=True, start_method="spawn")
    res = [torch.load(f"{out}.{r}", weights_only=True) for r in range(WORLD)]
    # replicas identical after the collective
    for k in ("params", "m", "v"):
        assert torch.equal(res[0][k], res[1][k]), k
    # == one process over the union batch
    s, a, r, s1, w, tw, m, v = _global_batch()
    ref = O.td_step(w, tw, m, v, 3, s, a, r, s1)
    np.testing.assert_allclose(res[0]["loss"], ref["loss"], rtol=1e-5)
    np.testing.assert_allclose(res[0]["norm"], ref["total_norm"], rtol=1e-5)
    np.testing.assert_allclose(res[0]["params"].numpy(), ref["params"].numpy(), rtol=0, atol=2e-6)
    np.testing.assert_allclose(res[0]["m"].numpy(), ref["m"].numpy(), rtol=1e-4, atol=1e-9)


class _FakePeerLib:
    """Host-side stand-in for libswarm_hip's peer setup calls (no GPU here): buffers are fake
    addresses, handles carry the owner's rank; ``fail`` makes this rank's allocation fail.
    It refuses any launch: a rank whose setup failed must never start an exchange."""

    def __init__(self, rank, fail):
        self.rank, self.fail = rank, fail

    def swarm_peer_alloc(self, pp):
        if self.fail:
            return 2   # hipErrorOutOfMemory
        pp._obj.value = 0x1000 * (self.rank + 1)
        return 0

    def swarm_peer_ipc_handle(self, buf, h):
        import ctypes
        ctypes.memmove(h, bytes([self.rank + 1]) * len(h), len(h))
        return 0

    def swarm_peer_ipc_open(self, buf, pp):
        pp._obj.value = 0x100000 + bytes(buf)[0]
        return 0

    def swarm_peer_ipc_close(self, p):
        return 0

    def swarm_peer_free(self, p):
        return 0

    def swarm_peer_allreduce(self, *a):
        raise AssertionError("an exchange was launched after a failed setup")


def _peer_setup_main(rank, port, out_path, fail_rank):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD))
    torch.set_num_threads(1)
    import swarm_amd._lib as L
    L.load = lambda *a, **k: _FakePeerLib(rank, rank == fail_rank)
    pg = swdist.init_process_group("gloo")
    end = swdist.PeerExchange.connect(pg, device="cpu")
    ok = end.selftest()
    # bench.py's decision: a MIN all-reduce of the flags, the same on every rank
    flag = torch.tensor([1 if ok else 0], dtype=torch.int32)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    end.close()
    torch.save(dict(ok=ok, error=str(end.error), flag=int(flag.item())), f"{out_path}.{rank}")
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("fail_rank", [0, 1])
def test_peer_setup_failure_on_one_rank_keeps_collectives_matched(tmp_path, fail_rank):
    """one rank's swarm_peer_alloc fails.  Both ranks still complete connect() (the
    handle gather and the barrier are always entered), neither launches an exchange, and the
    MIN of the self-test flags is 0 on both: bench.py falls back to RCCL on every rank together
    instead of hanging in mismatched collectives."""
    out = str(tmp_path / "rank")
    mp.start_processes(_peer_setup_main, args=(_free_port(), out, fail_rank), nprocs=WORLD, join=True,
                       start_method="spawn")
    res = [torch.load(f"{out}.{r}", weights_only=True) for r in range(WORLD)]
    assert all(not x["ok"] and x["flag"] == 0 for x in res)
    assert "swarm_peer_alloc" in res[fail_rank]["error"]
    assert f"rank {fail_rank} could not set up" in res[1 - fail_rank]["error"]
