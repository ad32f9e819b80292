"""``GCN`` — the reference's Q-network class (src/training/train_gcn_dqn.py:50-70)
with an identical ``state_dict`` layout, so ``data/models/*.pth`` load unchanged:

    conv1.att_src [1,1,32]  conv1.att_dst [1,1,32]  conv1.bias [32]
    conv1.lin.weight [32,7] lin1.weight [32,32] lin1.bias [32] lin2.weight [9,32] lin2.bias [9]

``forward(data)`` runs GATConv(7->32, heads=1, add_self_loops=False) -> tanh ->
lin1 -> relu -> lin2 for every graph of the batch in one HIP launch
(``swarm_q_forward``).  It is an inference forward (no autograd graph): the
learner's backward is the fused hand-written one in ``swarm_td_grad``.
``conv="gcn"`` selects the GCNConv variant (parity unpinned), which
reuses conv1.lin.weight / conv1.bias and ignores the attention vectors.

``GCN(7, 8, 9, layers=3)`` is the same class with its commented conv2/conv3 layers
(train_gcn_dqn.py:54-55, 65-68): conv1 -> tanh -> conv2 -> relu -> conv3 -> relu ->
lin1 -> relu -> lin2, hidden 8 — the architecture of the reference's Flocking checkpoints
(``data/models/experiment_Flocking-seed_*.pth``), forward only (``SWARM_NET_GAT3``).
``GCN.from_state_dict(sd)`` picks the architecture from the checkpoint's keys.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _lib
from ._lib import check, ptr, stream_ptr
from .engine import param_order
from .graph import Data, _lib_byref, _round4, edges_to_mult


class GATConvParams(nn.Module):
    """Parameter holder with PyG 2.5.3 GATConv's names and registration order."""

    def __init__(self, in_channels: int, out_channels: int):
        super().__init__()
        self.att_src = nn.Parameter(torch.empty(1, 1, out_channels))
        self.att_dst = nn.Parameter(torch.empty(1, 1, out_channels))
        self.bias = nn.Parameter(torch.zeros(out_channels))
        self.lin = nn.Linear(in_channels, out_channels, bias=False)
        for p in (self.att_src, self.att_dst):
            bound = (6.0 / (1 + out_channels)) ** 0.5
            nn.init.uniform_(p, -bound, bound)
        bound = (6.0 / (in_channels + out_channels)) ** 0.5
        nn.init.uniform_(self.lin.weight, -bound, bound)


class GCN(nn.Module):
    def __init__(self, input_dim: int = 7, hidden_dim: int = 32, output_dim: int = 9, conv: str = "gat",
                 layers: int = 1):
        super().__init__()
        shapes = {1: (7, 32, 9), 3: (7, 8, 9)}
        if shapes.get(layers) != (input_dim, hidden_dim, output_dim):
            raise ValueError("the HIP kernels are specialised for GCN(7, 32, 9) (train_gcn_dqn.py:81) and the "
                             "Flocking checkpoints' GCN(7, 8, 9, layers=3)")
        if layers == 3 and conv != "gat":
            raise ValueError("the three-layer network is a GAT")
        self.conv1 = GATConvParams(input_dim, hidden_dim)
        if layers == 3:
            self.conv2 = GATConvParams(hidden_dim, hidden_dim)
            self.conv3 = GATConvParams(hidden_dim, hidden_dim)
        self.lin1 = nn.Linear(hidden_dim, hidden_dim)
        self.lin2 = nn.Linear(hidden_dim, output_dim)
        self.conv = conv
        self.layers = layers
        self.net = "gat3" if layers == 3 else "gcn"
        self.net_id = _lib.NET_GAT3 if layers == 3 else _lib.NET_GCN
        self._flat = None
        self._flat_key = None

    @classmethod
    def from_state_dict(cls, sd, conv: str = "gat") -> "GCN":
        """A model of the checkpoint's architecture (three GATConvs if it holds conv2), loaded."""
        m = cls(7, 8, 9, conv, layers=3) if "conv2.lin.weight" in sd else cls(7, 32, 9, conv)
        m.load_state_dict(sd)
        return m

    def flat_params(self, device="cuda") -> torch.Tensor:
        sd = dict(self.named_parameters())
        order = param_order(self.net)
        key = tuple((id(sd[k]), sd[k]._version) for k, _ in order) + (str(device),)
        if self._flat is None or self._flat_key != key:
            self._flat = torch.cat([sd[k].detach().reshape(-1) for k, _ in order]).to(device, torch.float32)
            self._flat_key = key
        return self._flat

    def forward(self, data: Data) -> torch.Tensor:
        lib = _lib.load()
        x = data.x.to("cuda", torch.float32).contiguous()
        conv = _lib.CONV_GAT if self.conv == "gat" else _lib.CONV_GCN
        params = self.flat_params(x.device)
        M = x.shape[0]
        q = torch.empty(M, 9, dtype=torch.float32, device=x.device)
        if data.swarm is not None:
            m = data.swarm
            cfg = _lib.SwarmConfig(m["n_graphs"], m["n_nodes"], 0, m["graph"], m["k"], conv, 0, 0, 0,
                                   float(m.get("radius", 0.0)), self.net_id)
            check(lib.swarm_q_forward(_lib_byref(cfg), ptr(params), ptr(x), None, ptr(q), stream_ptr()),
                  "swarm_q_forward")
        else:
            G = data.num_graphs
            if M % G:
                raise ValueError("GCN.forward: graphs of unequal size are not supported")
            N = M // G
            mult = edges_to_mult(data.edge_index, G, N)
            cfg = _lib.SwarmConfig(G, N, 0, _lib.GRAPH_DENSE, 0, conv, 0, 0, 0, 0.0, self.net_id)
            check(lib.swarm_q_forward(_lib_byref(cfg), ptr(params), ptr(x), ptr(mult), ptr(q), stream_ptr()),
                  "swarm_q_forward")
        return q


__all__ = ["GCN", "GATConvParams", "_round4"]
