"""``go_to_position_scenario`` by module name (the reference's src/scenarios/go_to_position_scenario.py): ``GoToPositionScenario``
is this repository's scenario, whose world runs in libswarm_hip.so (reset, step, reward,
observation on the GPU)."""
import os as _os
import sys as _sys

_ROOT = _os.path.dirname(_os.path.dirname(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))))   # the repository root (swarm_amd)
if _ROOT not in _sys.path:
    _sys.path.append(_ROOT)

from swarm_amd import GoToPositionScenario  # noqa: E402,F401

__all__ = ["GoToPositionScenario"]
