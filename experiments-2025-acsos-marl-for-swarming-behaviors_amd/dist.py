"""Rank sharding and the one data-path collective of the training tick.

* Environments shard contiguously: rank r of W owns the global envs
  [r*B, (r+1)*B).  ``swarm_config.env_offset = r*B`` keys every Philox draw
  (reset centre, ε coin, random actions, replay sampling) by the GLOBAL env
  index, so env e evolves identically whatever the rank layout.
* Each rank keeps its own replay ring and samples S graphs from it.
* The only exchange is a SUM all-reduce of the flat gradient buffer
  (1,673 parameters + the loss sum) once per TD update; every rank then applies
  clip_grad_norm_ + Adam to grad / W (``swarm_adam_cfg.world_size``), so the
  replicas stay bit-identical.  The loss is a mean over nodes, hence with equal
  per-rank S this is the single-process update over the union batch
  (tests/test_dist_gloo.py checks it with the oracle on two gloo ranks).

One process per GPU; on ROCm the ``nccl`` backend of torch.distributed is RCCL
(xGMI between the GPUs of a node).  The 6.7 KB message is latency-bound: one
call per update, issued on the compute stream.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional

import torch


@dataclass(frozen=True)
class Shard:
    rank: int
    world_size: int
    envs_per_rank: int

    @property
    def env_offset(self) -> int:
        return self.rank * self.envs_per_rank

    @property
    def global_envs(self) -> int:
        return self.world_size * self.envs_per_rank

    def env_range(self) -> range:
        return range(self.env_offset, self.env_offset + self.envs_per_rank)


def shard_from_env(envs_per_rank: int) -> Shard:
    """Shard of this process from torchrun's RANK / WORLD_SIZE (1 rank if unset)."""
    return Shard(int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), envs_per_rank)


def init_process_group(backend: str, local_rank: Optional[int] = None):
    """torch.distributed.init_process_group for a torchrun launch (MASTER_ADDR 127.0.0.1)."""
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    kw = {}
    if backend == "nccl" and local_rank is not None:
        kw["device_id"] = torch.device("cuda", local_rank)
    dist.init_process_group(backend, **kw)
    return dist.group.WORLD


def allreduce_grad_(grad: torch.Tensor, world_size: int, group=None) -> torch.Tensor:
    """In-place SUM of the flat gradient over ranks (no-op for one rank without a group).
    The division by W happens inside the optimizer step (swarm_adam_cfg.world_size)."""
    if world_size > 1 or group is not None:
        import torch.distributed as dist
        dist.all_reduce(grad, op=dist.ReduceOp.SUM, group=group)
    return grad
