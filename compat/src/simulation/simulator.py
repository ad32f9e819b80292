"""``simulator`` by module name (the reference's src/simulation/simulator.py): ``Simulator``
(:28-166) and the module-level ``create_graph_from_observations(self, observations,
num_agents)`` (:9-26: each agent's 10 nearest by ``torch.topk`` over the fp32 distance, both
edge directions, plus [0, 0]), backed by the MI355X path.  ``Simulator`` runs each episode as
one rollout launch on the GPU (kNN build -> GAT -> argmax -> env.step per tick) and writes the
reference's CSV layout.  k defaults to the code's 10; the reference's recorded data used 5
(SURVEY §4), pass ``knn_k=5`` for that.
"""
import os as _os
import sys as _sys

_ROOT = _os.path.dirname(_os.path.dirname(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))))
if _ROOT not in _sys.path:
    _sys.path.append(_ROOT)

from swarm_amd import DQNTrainer, Simulator, create_knn_graph_from_observations  # noqa: E402,F401

__all__ = ["Simulator", "create_graph_from_observations", "DQNTrainer"]

KNN_K = 10   # simulator.py:19


def create_graph_from_observations(self, observations, num_agents):
    """simulator.py:9-26 (``self`` is unused there too): a kNN-10 graph over the agents of
    ``observations`` ({agent_i: [B, 6]}); the neighbour sets are built on the GPU with
    torch.topk's tie semantics."""
    return create_knn_graph_from_observations(observations, num_agents, KNN_K)
