"""Graph containers and builders with the reference's call shapes.

``Data`` / ``Batch`` mirror the subset of torch_geometric the reference uses
(``Data(x=..., edge_index=...)``, ``Batch.from_data_list``; train_gcn_dqn.py:45,109).
Graphs built here carry a compact description (n_graphs, n_nodes, kind, k) so that
``GCN.forward`` hands the whole batch to one HIP launch; the explicit PyG
``edge_index`` is materialised only when someone reads it.

Builders:
* ``create_graph_from_observations(obs)`` — training graph, train_gcn_dqn.py:94-110:
  every ordered pair (i, j), i != j, plus one extra (0, 0) self loop.
* ``create_knn_graph_from_observations(obs, n_agents, k)`` — evaluation graph,
  simulator.py:9-26: per node its k nearest (torch.topk set semantics, itself
  included), edges both ways, plus (0, 0).
* ``create_radius_graph_from_observations(obs, n_agents, radius)`` — the north_star's
  radius-neighbour graph (not in the reference; SURVEY §8(f) row 3, parity unpinned):
  edge (i, j) for every j != i with |p_i - p_j| <= radius (the kNN build's fp32 distance),
  plus (0, 0) as both reference builders append it.
"""
from __future__ import annotations

from typing import Optional

import torch

from . import _lib
from ._lib import check, ptr, stream_ptr


class Data:
    def __init__(self, x: Optional[torch.Tensor] = None, edge_index: Optional[torch.Tensor] = None, *,
                 swarm: Optional[dict] = None, **kwargs):
        self.x = x
        self._edge_index = edge_index
        self.swarm = swarm          # dict(n_graphs, n_nodes, graph, k) for builder-made graphs
        for k, v in kwargs.items():
            setattr(self, k, v)

    @property
    def edge_index(self) -> torch.Tensor:
        if self._edge_index is None and self.swarm is not None:
            self._edge_index = edge_index_from_mult(build_mult(self))
        return self._edge_index

    @edge_index.setter
    def edge_index(self, v):
        self._edge_index = v

    @property
    def num_nodes(self) -> int:
        return 0 if self.x is None else int(self.x.shape[0])

    @property
    def num_graphs(self) -> int:
        return self.swarm["n_graphs"] if self.swarm else getattr(self, "_num_graphs", 1)

    def to(self, device):
        d = Data(self.x.to(device) if self.x is not None else None,
                 self._edge_index.to(device) if self._edge_index is not None else None, swarm=self.swarm)
        return d


class Batch(Data):
    @staticmethod
    def from_data_list(data_list):
        xs = [d.x for d in data_list]
        x = torch.cat(xs, dim=0)
        metas = [d.swarm for d in data_list]
        if all(m is not None for m in metas) and len({(m["n_nodes"], m["graph"], m["k"], m.get("radius", 0.0))
                                                      for m in metas}) == 1:
            m = dict(metas[0])
            m["n_graphs"] = sum(mm["n_graphs"] for mm in metas)
            b = Batch(x, None, swarm=m)
        else:
            eis, off = [], 0
            for d in data_list:
                eis.append(d.edge_index + off)
                off += d.num_nodes
            b = Batch(x, torch.cat(eis, dim=1))
        b._num_graphs = len(data_list)
        return b


def _node_features(observations) -> torch.Tensor:
    """{agent_i: [B, 6]} (or [B, N, 6]) -> x [B*N, 7] = [obs, float(i)], env-major."""
    if isinstance(observations, dict):
        n = len(observations)
        obs = torch.stack([observations[f"agent{i}"] for i in range(n)], dim=1)   # [B, N, 6]
    else:
        obs = observations
    B, N, _ = obs.shape
    ids = torch.arange(N, dtype=obs.dtype, device=obs.device).view(1, N, 1).expand(B, N, 1)
    return torch.cat([obs, ids], dim=-1).reshape(B * N, 7)


def create_graph_from_observations(observations) -> Data:
    x = _node_features(observations)
    n = len(observations) if isinstance(observations, dict) else observations.shape[1]
    return Data(x, None, swarm=dict(n_graphs=x.shape[0] // n, n_nodes=n, graph=_lib.GRAPH_COMPLETE, k=0))


def create_knn_graph_from_observations(observations, num_agents: int, k: int = 10) -> Data:
    if k > num_agents:
        raise RuntimeError("selected index k out of range")
    x = _node_features(observations)
    return Data(x, None, swarm=dict(n_graphs=x.shape[0] // num_agents, n_nodes=num_agents, graph=_lib.GRAPH_KNN, k=k))


def create_radius_graph_from_observations(observations, num_agents: int, radius: float) -> Data:
    if not radius > 0.0:
        raise ValueError("radius must be > 0")
    x = _node_features(observations)
    return Data(x, None, swarm=dict(n_graphs=x.shape[0] // num_agents, n_nodes=num_agents, graph=_lib.GRAPH_RADIUS,
                                    k=0, radius=float(radius)))


def graph_config(data: Data, scenario: int = 0, conv: int = _lib.CONV_GAT) -> _lib.SwarmConfig:
    m = data.swarm
    return _lib.SwarmConfig(m["n_graphs"], m["n_nodes"], scenario, m["graph"], m["k"], conv, 0, 0, 0,
                            float(m.get("radius", 0.0)), 0)


def build_mult(data: Data) -> torch.Tensor:
    """Dense multiplicity [G, N, N] (uint8, mult[g,u,v] = #edges u->v) on the GPU."""
    lib = _lib.load()
    x = data.x.to("cuda", torch.float32).contiguous()
    if data.swarm is not None:
        m = data.swarm
        mult = torch.zeros(_round4(m["n_graphs"] * m["n_nodes"] ** 2), dtype=torch.uint8, device=x.device)
        cfg = graph_config(data)
        check(lib.swarm_build_graph(_lib_byref(cfg), ptr(x), ptr(mult), stream_ptr()), "swarm_build_graph")
        return mult[: m["n_graphs"] * m["n_nodes"] ** 2].view(m["n_graphs"], m["n_nodes"], m["n_nodes"])
    G = data.num_graphs
    N = data.num_nodes // G
    return edges_to_mult(data.edge_index, G, N)


def edges_to_mult(edge_index: torch.Tensor, n_graphs: int, n_nodes: int) -> torch.Tensor:
    lib = _lib.load()
    ei = edge_index.to("cuda", torch.int64).contiguous()
    mult = torch.zeros(_round4(n_graphs * n_nodes * n_nodes), dtype=torch.uint8, device=ei.device)
    err = torch.zeros(1, dtype=torch.int32, device=ei.device)
    check(lib.swarm_edges_to_mult(ptr(ei), ei.shape[1], n_graphs, n_nodes, ptr(mult), ptr(err), stream_ptr()),
          "swarm_edges_to_mult")
    if int(err.item()) != 0:
        raise ValueError("edge_index has an edge between different graphs (expected Batch of equal-size graphs)")
    return mult[: n_graphs * n_nodes * n_nodes].view(n_graphs, n_nodes, n_nodes)


def edge_index_from_mult(mult: torch.Tensor) -> torch.Tensor:
    """Inspection helper: dense multiplicity -> PyG edge_index (edges grouped by target)."""
    G, N, _ = mult.shape
    m = mult.to(torch.int64)
    g, u, v = torch.nonzero(m, as_tuple=True)
    reps = m[g, u, v]
    src = torch.repeat_interleave(g * N + u, reps)
    dst = torch.repeat_interleave(g * N + v, reps)
    return torch.stack([src, dst])


def _round4(n: int) -> int:
    return (n + 3) & ~3


def _lib_byref(obj):
    import ctypes
    return ctypes.byref(obj)
