"""MI355X-native hot path of davidedomini/experiments-2025-acsos-marl-for-swarming-behaviors.

Import as ``swarm_amd`` (the top-level shim ``swarm_amd.py`` maps that name to
this directory).  Public surface mirrors the reference:

    from swarm_amd import make_env, GoToPositionScenario, ObstacleAvoidanceScenario
    from swarm_amd import GCN, DQNTrainer, GraphReplayBuffer, Simulator, set_seed, get_scenario
    from swarm_amd import SwarmEngine          # the fused device engine underneath

The compute path is libswarm_hip.so (csrc/, C ABI in include/swarm_hip.h); there
is no CPU fallback.
"""
from ._lib import load as load_library  # noqa: F401
from .engine import SwarmEngine, flatten_state_dict, unflatten_params  # noqa: F401
from .graph import (Batch, Data, create_graph_from_observations, create_knn_graph_from_observations,  # noqa: F401
                    create_radius_graph_from_observations)
from .gcn import GCN  # noqa: F401
from .scenarios import (BaseScenario, FlockingScenario, GoToPositionScenario, ObstacleAvoidanceScenario,  # noqa: F401
                        get_scenario)
from .env import Environment, make_env  # noqa: F401
from .dqn import DQNTrainer, GraphReplayBuffer, set_seed  # noqa: F401
from .simulator import Simulator  # noqa: F401

__all__ = ["SwarmEngine", "Data", "Batch", "GCN", "make_env", "Environment", "GoToPositionScenario",
           "ObstacleAvoidanceScenario", "FlockingScenario", "BaseScenario", "get_scenario", "DQNTrainer", "GraphReplayBuffer",
           "set_seed", "Simulator", "create_graph_from_observations", "create_knn_graph_from_observations",
           "create_radius_graph_from_observations"]
