"""The reference's experiment scripts run by module name (VERDICT r2 "next" #6).

``compat/`` mirrors the reference's layout (``vmas``, ``src/scenarios``, ``src/training``,
``src/simulation``), so the scripts' own import lines resolve to this repository:

    from vmas import make_env                                    tests/test_go_to_position.py:4
    sys.path.insert(..., '../src/{scenarios,training,simulation}')                     :7-13
    from train_gcn_dqn import GCN                                                      :15
    from go_to_position_scenario import GoToPositionScenario                           :16
    from simulator import Simulator                                                    :17

The GPU test writes a script with exactly those imports and the script's call sequence
(make_env -> GCN(7, 32, 9).load_state_dict(torch.load(...)) -> Simulator(...).run_simulation(),
:29-53) for one model seed at agents 10 and 11, runs it from a directory laid out like the
reference checkout (src/ -> compat/src, data/models/ holding the fixture weights as .pth), and
checks its CSV outputs against this package's own Simulator on the same inputs.
"""
import csv
import importlib
import os
import runpy
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COMPAT = os.path.join(ROOT, "compat")

SCRIPT = '''\
import sys
import os
from vmas import make_env
import torch

scenarios_dir = os.path.abspath(os.path.join(os.path.dirname(__file__), '..', 'src', 'scenarios'))
training_dir = os.path.abspath(os.path.join(os.path.dirname(__file__), '..', 'src', 'training'))
simulation_dir = os.path.abspath(os.path.join(os.path.dirname(__file__), '..', 'src', 'simulation'))

sys.path.insert(0, scenarios_dir)
sys.path.insert(1, training_dir)
sys.path.insert(2, simulation_dir)

from train_gcn_dqn import GCN
from {module} import {cls}
from simulator import Simulator

if __name__ == "__main__":
    models_seed = [{seed}]
    simulation_seed = 6967
    agents = {agents}

    for model_seed in models_seed:
        for agent in agents:
            env = make_env(
                {cls}(),
                scenario_name="test_gcn_vmas",
                num_envs=1,
                device="cpu",
                continuous_actions=False,
                dict_spaces=True,
                wrapper=None,
                seed=simulation_seed,
                n_agents=agent,
                max_steps={max_steps},
                random=True,
            )
            models_dir = "data/models/"
            model = GCN(input_dim=7, hidden_dim=32, output_dim=9)
            model.load_state_dict(torch.load(models_dir + f'experiment_{experiment}-seed_{{model_seed}}.pth'))
            model.eval()
            simulator = Simulator(env, model, 8, '{name}', simulation_seed,
                                  output_dir=f'data/test_stats/{name}/seed_{{model_seed}}/agents_{{agent}}')
            simulator.run_simulation()
'''

CASES = {"go_to": ("go_to_position_scenario", "GoToPositionScenario", "GoTo", 50),
         "obstacle_avoidance": ("obstacle_avoidance_scenario", "ObstacleAvoidanceScenario", "ObstacleAvoidance", 100)}
MODULES = ("vmas", "train_gcn_dqn", "simulator", "go_to_position_scenario", "obstacle_avoidance_scenario",
           "flocking_scenario")


def _compat_imports():
    """Import the compat modules the way the scripts do (their directories on sys.path)."""
    saved = list(sys.path)
    sys.path[:0] = [COMPAT, os.path.join(COMPAT, "src", "scenarios"), os.path.join(COMPAT, "src", "training"),
                    os.path.join(COMPAT, "src", "simulation")]
    try:
        return {m: importlib.import_module(m) for m in MODULES}
    finally:
        sys.path[:] = saved
        for m in MODULES:
            sys.modules.pop(m, None)


def test_compat_modules_expose_the_reference_names():
    """CPU: every name the reference's scripts and modules import resolves (no GPU call)."""
    import inspect
    import swarm_amd
    mods = _compat_imports()
    assert mods["vmas"].make_env is swarm_amd.make_env
    t = mods["train_gcn_dqn"]
    for name in ("GCN", "DQNTrainer", "GraphReplayBuffer", "set_seed", "get_scenario"):
        assert getattr(t, name) is getattr(swarm_amd, name)
    assert callable(t.main)
    s = mods["simulator"]
    assert s.Simulator is swarm_amd.Simulator and s.DQNTrainer is swarm_amd.DQNTrainer
    assert list(inspect.signature(s.create_graph_from_observations).parameters) == ["self", "observations", "num_agents"]
    assert s.KNN_K == 10   # simulator.py:19
    assert mods["go_to_position_scenario"].GoToPositionScenario is swarm_amd.GoToPositionScenario
    assert mods["obstacle_avoidance_scenario"].ObstacleAvoidanceScenario is swarm_amd.ObstacleAvoidanceScenario
    assert mods["flocking_scenario"].FlockingScenario is swarm_amd.FlockingScenario
    sd = t.GCN(input_dim=7, hidden_dim=32, output_dim=9).state_dict()
    assert list(sd) == ["conv1.att_src", "conv1.att_dst", "conv1.bias", "conv1.lin.weight", "lin1.weight", "lin1.bias",
                        "lin2.weight", "lin2.bias"]


def _read(path):
    with open(path) as f:
        return list(csv.reader(f))


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["go_to", "obstacle_avoidance"])
def test_reference_script_runs_by_module_name(golden_weights, tmp_path, name, monkeypatch):
    import swarm_amd
    from oracle import swarm_oracle as O
    module, cls, experiment, max_steps = CASES[name]
    seed, agents = 0, [10, 11]
    (tmp_path / "tests").mkdir()
    (tmp_path / "src").symlink_to(os.path.join(COMPAT, "src"))
    models = tmp_path / "data" / "models"
    models.mkdir(parents=True)
    torch.save(O.unflatten_params(torch.tensor(golden_weights[name][seed])), models / f"experiment_{experiment}-seed_{seed}.pth")
    script = tmp_path / "tests" / f"test_{name}.py"
    script.write_text(SCRIPT.format(module=module, cls=cls, seed=seed, agents=agents, max_steps=max_steps,
                                    experiment=experiment, name=name))
    monkeypatch.chdir(tmp_path)
    monkeypatch.setattr(sys, "path", [COMPAT] + list(sys.path))
    try:
        runpy.run_path(str(script), run_name="__main__")
    finally:
        for m in MODULES:
            sys.modules.pop(m, None)
    for n in agents:
        out = tmp_path / "data" / "test_stats" / name / f"seed_{seed}" / f"agents_{n}"
        rows = _read(out / "result.csv")
        assert rows[0] == ["Episode", "Reward", "Collisions", "Distance (end)", "Distance (beginning)"]
        assert len(rows) == 9
        pos = _read(out / "positions" / "positions_episode_7_x.csv")
        assert len(pos) == max_steps + 1 and len(pos[0]) == n + 1
        # the same evaluation through the package directly: identical CSVs
        env = swarm_amd.make_env(getattr(swarm_amd, cls)(), num_envs=1, continuous_actions=False, dict_spaces=True,
                                 seed=6967, n_agents=n, max_steps=max_steps, random=True)
        model = swarm_amd.GCN(7, 32, 9)
        model.load_state_dict(torch.load(models / f"experiment_{experiment}-seed_{seed}.pth", weights_only=True))
        direct = tmp_path / "direct" / str(n)
        swarm_amd.Simulator(env, model, 8, name, 6967, output_dir=str(direct), knn_k=10).run_simulation()
        assert _read(direct / "result.csv") == rows
        assert _read(direct / "positions" / "positions_episode_7_x.csv") == pos
