"""Scenario plugins with the reference's class names and ``make_world`` kwargs.

In the reference these are VMAS ``BaseScenario`` subclasses whose
``reset_world_at`` / ``reward`` / ``observation`` VMAS calls on every step
(src/scenarios/go_to_position_scenario.py, src/scenarios/obstacle_avoidance_scenario.py,
src/scenarios/flocking_scenario.py).
Here the arithmetic of those methods lives in the HIP kernels
(``csrc/swarm_env.h`` agent_step / oa_reward, ``csrc/swarm_act.hip`` reset);
the classes carry the configuration and expose the metric helpers the
reference's callers use (``average_distance_to_goal``, ``obstacles_hits``,
``average_distance_to_obstacles``; simulator.py:62-87), computed from the
device-resident step outputs of the environment they are bound to.
"""
from __future__ import annotations

import torch

from . import _lib

GOAL = (-0.8, 0.8)
OBSTACLE = (-0.1, 0.1)


class BaseScenario:
    """Plugin interface (VMAS BaseScenario subset used by the reference)."""

    SCENARIO_ID = None
    env = None

    def make_world(self, batch_dim: int, device, **kwargs):
        self.batch_dim = batch_dim
        self.device = device
        self.n_agents = kwargs.get("n_agents", 1)
        self.seed = kwargs.get("seed", 1)
        self.kwargs = kwargs
        return self

    # per-agent views of the last step (VMAS calls these internally)
    def observation(self, agent):
        return self.env._last_obs[:, self._idx(agent)]

    def reward(self, agent):
        return self.env.engine.reward[:, self._idx(agent)]

    def done(self):
        return torch.zeros(self.batch_dim, dtype=torch.bool, device=self.env.engine.device)

    def info(self, agent):
        z = torch.zeros(self.batch_dim, device=self.env.engine.device)
        return {"pos_rew": z, "final_rew": z}

    def reset_world_at(self, env_index=None):
        self.env.reset()

    def _idx(self, agent):
        name = agent if isinstance(agent, str) else agent.name
        return int(name.replace("agent", ""))

    # metric helpers (0-dim tensors like the reference; B envs are pooled)
    def average_distance_to_goal(self):
        return self.env.engine.avg_dist.mean()

    def average_distance_to_goal_per_env(self):
        return self.env.engine.avg_dist

    def obstacles_hits(self):
        return torch.tensor(0.0)

    def average_distance_to_obstacles(self):
        return torch.tensor(0.0)


class GoToPositionScenario(BaseScenario):
    """go_to_position_scenario.py: goal (-0.8, 0.8), collective reward -sum_j |p_j - goal|,
    reset centre (1.5,-1.5) + N((-0.6,0.6), 0.4) shared by every env (:83-106)."""

    SCENARIO_ID = _lib.SWARM_GOTO

    def make_world(self, batch_dim, device, **kwargs):
        super().make_world(batch_dim, device, **kwargs)
        self.pos_shaping_factor = kwargs.get("pos_shaping_factor", 1.0)
        self.agent_radius = kwargs.get("agent_radius", 0.1)   # unused by the physics (VMAS sphere r=0.05)
        self.random = True
        return self


class ObstacleAvoidanceScenario(BaseScenario):
    """obstacle_avoidance_scenario.py: obstacle (-0.1, 0.1) r=0.05, reward
    -d_goal + 2.5 * (d_obs <= 1 ? -(1 - d_obs) : 0), hits = #[d_obs <= 0.2];
    reset centre (0.6,-0.6) + (random ? N(0, 0.1) : 0) (:94-133; the centre :100-102)."""

    SCENARIO_ID = _lib.SWARM_OBSTACLE_AVOIDANCE

    def make_world(self, batch_dim, device, **kwargs):
        super().make_world(batch_dim, device, **kwargs)
        self.random = kwargs.get("random", False)
        self.pos_shaping_factor = kwargs.get("pos_shaping_factor", 10.0)
        self.dist_shaping_factor = kwargs.get("dist_shaping_factor", 10.0)
        self.n_obstacles = 1
        self.min_collision_distance_reward = 1
        self.min_collision_distance_count = 0.2
        return self

    def obstacles_hits(self):
        return self.env.engine.hits.sum()

    def obstacles_hits_per_env(self):
        return self.env.engine.hits

    def average_distance_to_obstacles(self):
        pos = self.env.engine.state[..., :2]
        d = torch.linalg.vector_norm(pos - torch.tensor(OBSTACLE, device=pos.device), dim=-1) - 0.05 - 0.05
        return d.mean()


class FlockingScenario(BaseScenario):
    """flocking_scenario.py: goal (-0.8, 0.8); collective reward, summed over agents, of the
    shaped goal progress (x10, +50 on the goal), -1 per agent in contact
    (World.get_distance <= 0.005) and the shaped change of the mean squared deviation
    from the desired spacing 0.15 (x10); reset centre [-1, 1] + N((-0.6,0.6), 0.4)
    shared by every env (:9-176).  The kernel holds the scenario's constants, so only
    the reference's defaults are accepted."""

    SCENARIO_ID = _lib.SWARM_FLOCKING

    def make_world(self, batch_dim, device, **kwargs):
        super().make_world(batch_dim, device, **kwargs)
        self.pos_shaping_factor = kwargs.get("pos_shaping_factor", 10.0)
        self.dist_shaping_factor = kwargs.get("dist_shaping_factor", 10.0)
        self.agent_radius = kwargs.get("agent_radius", 0.1)   # unused by the physics (VMAS sphere r=0.05)
        if self.pos_shaping_factor != 10.0 or self.dist_shaping_factor != 10.0:
            raise NotImplementedError("FlockingScenario: the kernels hold the reference's shaping factors (10, 10)")
        if self.n_agents < 2:
            raise ValueError("FlockingScenario needs n_agents >= 2 (its spacing reward averages over the others)")
        self.desired_distance = 0.15
        self.min_collision_distance = 0.005
        self.agent_collision_reward = -1
        self.random = True
        return self

    def distance_to_goal_all(self):
        """flocking_scenario.py:188-195: [B, N] distances to the goal."""
        pos = self.env.engine.state[..., :2]
        return torch.linalg.vector_norm(pos - torch.tensor(GOAL, device=pos.device), dim=-1)

    def agent_contacts(self):
        """Agents in contact after the last step, summed over agents and envs (the count
        behind the scenario's -1 avoidance terms)."""
        return self.env.engine.hits.sum()


def get_scenario(experiment_name: str) -> BaseScenario:
    """train_gcn_dqn.py:241-249."""
    if experiment_name == "GoTo":
        return GoToPositionScenario()
    if experiment_name == "ObstacleAvoidance":
        return ObstacleAvoidanceScenario()
    if experiment_name == "Flocking":
        return FlockingScenario()
    raise Exception(f"Scenario {experiment_name} not supported! Please check :)")
