"""``train_gcn_dqn`` by module name (the reference's src/training/train_gcn_dqn.py): the names
the reference's scripts import from it, backed by the MI355X path.

    GCN                  train_gcn_dqn.py:50-70   (same state_dict keys; data/models/*.pth load)
    GraphReplayBuffer    :25-48
    DQNTrainer           :72-231  (create_graph_from_observations, train_step_dqn, train_model,
                                   save_metrics_to_csv; the episode loop runs fused on the GPU)
    set_seed             :233-239
    get_scenario         :241-249

Run as a script it is the reference's training driver (:252-292): seeds 0-9 x
['ObstacleAvoidance', 'GoTo'], 10 agents, 1 env, 1000 episodes of 100 ticks, models to
data/models/, learning curves to data/stats/.
"""
import os as _os
import sys as _sys

_ROOT = _os.path.dirname(_os.path.dirname(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))))
if _ROOT not in _sys.path:
    _sys.path.append(_ROOT)

from swarm_amd import GCN, DQNTrainer, GraphReplayBuffer, get_scenario, make_env, set_seed  # noqa: E402,F401

__all__ = ["GCN", "DQNTrainer", "GraphReplayBuffer", "set_seed", "get_scenario", "main"]


def main(max_seed=10, experiments=("ObstacleAvoidance", "GoTo"), agents=10, episodes=1000,
         models_path="data/models/", stats_path="data/stats/"):
    """The reference's __main__ block (train_gcn_dqn.py:252-292), parameterised."""
    from pathlib import Path
    for p in (stats_path, "data/test_stats/", models_path):
        Path(p).mkdir(parents=True, exist_ok=True)
    config = {"epsilon": 0.99, "epsilon_decay": 0.01, "min_epsilon": 0.05, "episodes": episodes}
    for seed in range(max_seed):
        set_seed(seed)
        for experiment in experiments:
            print(f"Running seed {seed} experiment {experiment}")
            env = make_env(scenario=get_scenario(experiment), num_envs=1, device="cpu", continuous_actions=False,
                           wrapper=None, max_steps=100, dict_spaces=True, n_agents=agents, seed=seed)
            trainer = DQNTrainer(env, seed, models_path, stats_path, experiment)
            trainer.train_model(config)


if __name__ == "__main__":
    main()
