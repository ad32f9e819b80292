"""The reference's experiment scripts resolve to this package by module name (VERDICT r2 "next" #6).

``compat/`` mirrors the reference checkout's layout (``vmas``, ``src/scenarios``, ``src/training``,
``src/simulation``): with those directories on ``sys.path``, as the reference's evaluation scripts
put them there (tests/test_go_to_position.py:7-13), ``vmas.make_env``, ``train_gcn_dqn.GCN``,
``simulator.Simulator`` and the scenario modules import from this repository.

The GPU test imports the compat modules by name and drives the evaluation call sequence the
scripts use (make_env -> GCN(7, 32, 9) -> load_state_dict(torch.load(.pth)) -> Simulator ->
run_simulation, with the scripts' seed 6967 and output layout) in its own code, then checks the
CSV outputs against this package's Simulator called directly on the same inputs.  No reference
script text is stored or executed here.
"""
import csv
import importlib
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COMPAT = os.path.join(ROOT, "compat")

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


def _evaluate_through_compat(mods, module, cls, experiment, name, seed, agents, max_steps, models, out_root):
    """The evaluation scripts' call sequence, through the compat modules: one Simulator run of 8
    episodes per agent count, outputs under out_root/<name>/seed_<seed>/agents_<n>."""
    scenario_cls = getattr(mods[module], cls)
    for n in agents:
        env = mods["vmas"].make_env(scenario_cls(), scenario_name="test_gcn_vmas", num_envs=1, device="cpu",
                                    continuous_actions=False, dict_spaces=True, wrapper=None, seed=6967, n_agents=n,
                                    max_steps=max_steps, random=True)
        net = mods["train_gcn_dqn"].GCN(input_dim=7, hidden_dim=32, output_dim=9)
        net.load_state_dict(torch.load(os.path.join(models, f"experiment_{experiment}-seed_{seed}.pth"),
                                       weights_only=True))
        net.eval()
        sim = mods["simulator"].Simulator(env, net, 8, name, 6967,
                                          output_dir=os.path.join(out_root, name, f"seed_{seed}", f"agents_{n}"))
        sim.run_simulation()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["go_to", "obstacle_avoidance"])
def test_reference_call_sequence_runs_by_module_name(golden_weights, tmp_path, name, monkeypatch):
    import swarm_amd
    from oracle import swarm_oracle as O
    module, cls, experiment, max_steps = CASES[name]
    seed, agents = 0, [10, 11]
    models = tmp_path / "data" / "models"
    models.mkdir(parents=True)
    torch.save(O.unflatten_params(torch.tensor(golden_weights[name][seed])), models / f"experiment_{experiment}-seed_{seed}.pth")
    monkeypatch.chdir(tmp_path)
    saved = list(sys.path)
    sys.path[:0] = [COMPAT, os.path.join(COMPAT, "src", "scenarios"), os.path.join(COMPAT, "src", "training"),
                    os.path.join(COMPAT, "src", "simulation")]
    try:
        mods = {m: importlib.import_module(m) for m in ("vmas", "train_gcn_dqn", "simulator", module)}
        _evaluate_through_compat(mods, module, cls, experiment, name, seed, agents, max_steps, str(models),
                                 str(tmp_path / "data" / "test_stats"))
    finally:
        sys.path[:] = saved
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
