"""``make_env`` / ``Environment`` with the VMAS 1.4.0 surface the reference uses
(train_gcn_dqn.py:79-80,149-171; simulator.py:50-93; tests/test_go_to_position.py:29-40):

    env = make_env(scenario, num_envs, device, continuous_actions=False, wrapper=None,
                   max_steps, dict_spaces=True, seed, n_agents, random, scenario_name)
    obs = env.reset()                         # {agent_i: [B, 6]}
    obs, rews, dones, infos = env.step({agent_i: [B] int})
    env.n_agents, env.agents, env.max_steps, env.device, env.scenario,
    env.observation_space['agent0'].shape[0] == 6, env.action_space['agent0'].n == 9

Everything runs on the GPU (``swarm_env_reset`` / ``swarm_env_step``); returned
tensors live on the GPU whatever ``device`` was requested.
"""
from __future__ import annotations

from types import SimpleNamespace

import torch

from .engine import SwarmEngine
from .scenarios import GOAL, BaseScenario


class _Box:
    def __init__(self, shape):
        self.shape = shape


class _Discrete:
    def __init__(self, n):
        self.n = n


class Agent(SimpleNamespace):
    pass


class Environment:
    def __init__(self, scenario: BaseScenario, num_envs: int = 1, device="cuda", max_steps=None, seed=None,
                 dict_spaces: bool = True, continuous_actions: bool = False, **kwargs):
        if continuous_actions:
            raise NotImplementedError("only discrete actions (continuous_actions=False) are supported")
        self.scenario = scenario
        self.num_envs = num_envs
        self.batch_dim = num_envs
        self.max_steps = max_steps
        self.dict_spaces = dict_spaces
        self.seed_value = 0 if seed is None else int(seed)
        self.requested_device = device
        kwargs.setdefault("seed", self.seed_value)
        scenario.make_world(num_envs, device, **kwargs)
        self.n_agents = scenario.n_agents
        self.engine = SwarmEngine(scenario=scenario.SCENARIO_ID, n_agents=self.n_agents, n_envs=num_envs,
                                  seed=self.seed_value, learn=False, shared_reset=True,
                                  random_oa=bool(getattr(scenario, "random", True)), eps=0.0)
        self.device = self.engine.device
        scenario.env = self
        self.agents = [Agent(name=f"agent{i}") for i in range(self.n_agents)]
        names = [a.name for a in self.agents]
        self.observation_space = {n: _Box((6,)) for n in names}
        self.action_space = {n: _Discrete(9) for n in names}
        self.steps = torch.zeros(num_envs, device=self.device)
        self._last_obs = None

    def _obs_from_state(self):
        st = self.engine.state
        goal = torch.tensor(GOAL, device=st.device).expand(st.shape[0], st.shape[1], 2)
        return torch.cat([st, goal], dim=-1)

    def _split(self, obs):
        if self.dict_spaces:
            return {f"agent{i}": obs[:, i] for i in range(self.n_agents)}
        return [obs[:, i] for i in range(self.n_agents)]

    def reset(self, seed=None, return_observations=True, return_info=False, return_dones=False):
        if seed is not None:
            self.engine.cfg.seed = int(seed)
        self.engine.reset()
        self.steps.zero_()
        self._last_obs = self._obs_from_state()
        return self._split(self._last_obs) if return_observations else None

    def step(self, actions):
        if isinstance(actions, dict):
            acts = [actions[f"agent{i}"] for i in range(self.n_agents)]
        else:
            acts = list(actions)
        a = torch.stack([torch.as_tensor(x).reshape(-1).to(self.device) for x in acts], dim=1)
        a = a.expand(self.num_envs, self.n_agents) if a.shape[0] == 1 else a
        self.engine.env_step(a)
        self.steps += 1
        self._last_obs = self.engine.obs.clone()
        rews = {f"agent{i}": self.engine.reward[:, i].clone() for i in range(self.n_agents)}
        dones = torch.zeros(self.num_envs, dtype=torch.bool, device=self.device)
        if self.max_steps is not None:
            dones = dones | (self.steps >= self.max_steps)
        infos = {f"agent{i}": self.scenario.info(self.agents[i]) for i in range(self.n_agents)}
        obs = self._split(self._last_obs)
        if not self.dict_spaces:
            rews = list(rews.values())
            infos = list(infos.values())
        return obs, rews, dones, infos

    def render(self, *args, **kwargs):
        raise NotImplementedError("rendering is out of scope (SURVEY §2)")


def make_env(scenario, num_envs: int = 32, device="cuda", continuous_actions: bool = True, wrapper=None,
             max_steps=None, seed=None, dict_spaces: bool = False, **kwargs) -> Environment:
    """vmas.make_env subset. ``scenario`` must be one of this package's scenario objects."""
    if wrapper is not None:
        raise NotImplementedError("wrappers are out of scope")
    kwargs.pop("scenario_name", None)
    return Environment(scenario, num_envs=num_envs, device=device, max_steps=max_steps, seed=seed,
                       dict_spaces=dict_spaces, continuous_actions=continuous_actions, **kwargs)
