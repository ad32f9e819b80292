"""Import shim: ``import swarm_amd`` loads the package directory
``experiments-2025-acsos-marl-for-swarming-behaviors_amd/`` (whose name is not a
valid Python identifier) under the module name ``swarm_amd``."""
import importlib.util
import os
import sys

_PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                        "experiments-2025-acsos-marl-for-swarming-behaviors_amd")
_spec = importlib.util.spec_from_file_location("swarm_amd", os.path.join(_PKG_DIR, "__init__.py"),
                                               submodule_search_locations=[_PKG_DIR])
_mod = importlib.util.module_from_spec(_spec)
sys.modules["swarm_amd"] = _mod
_spec.loader.exec_module(_mod)
