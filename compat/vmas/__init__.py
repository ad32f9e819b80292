"""``vmas`` by module name, for the reference's scripts (``from vmas import make_env``,
/root/reference tests/test_go_to_position.py:4, tests/test_obstacle_avoidance.py:4,
src/training/train_gcn_dqn.py:12).

The compat tree mirrors the reference's layout so its scripts run unmodified:

    compat/vmas/                         make_env (this module)
    compat/src/scenarios/*.py            the scenario classes, by their reference module names
    compat/src/training/train_gcn_dqn.py GCN, DQNTrainer, GraphReplayBuffer, set_seed, get_scenario
    compat/src/simulation/simulator.py   Simulator, create_graph_from_observations
    compat/tests/                        drop the reference's experiment scripts here

Run from ``compat/`` with ``PYTHONPATH=<repo>/compat``; the scripts' own ``sys.path`` inserts
(``../src/{scenarios,training,simulation}``) then resolve to these modules.  Everything
underneath is the MI355X path (``swarm_amd``: libswarm_hip.so, no CPU fallback).
"""
import os as _os
import sys as _sys

_ROOT = _os.path.dirname(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))   # the repository root (swarm_amd)
if _ROOT not in _sys.path:
    _sys.path.append(_ROOT)

from swarm_amd import make_env  # noqa: E402,F401
from swarm_amd.env import Environment  # noqa: E402,F401

__all__ = ["make_env", "Environment"]
