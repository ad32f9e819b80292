"""``DQNTrainer`` / ``GraphReplayBuffer`` with the reference's API
(src/training/train_gcn_dqn.py:25-231), driven by the fused device engine.

``train_model(config)`` runs the reference's episode loop (:139-204): per episode
reset, then ``max_steps`` fused training ticks (act -> env.step -> replay push ->
TD update -> target sync every ``update_target_every`` ticks), ε schedule
``max(min_epsilon, epsilon * exp(-epsilon_decay * episode))`` (:180), model saved
as ``experiment_{experiment}-seed_{seed}.pth`` (:201) and the stats CSV with the
reference's ``i // 10`` indexing (:225-231).  One episode is captured once into a
hipGraph and replayed.

Deliberate, documented differences (SURVEY §7 "RNG", "Vectorisation fixes"):
random draws come from Philox keyed by (seed, tick, env), not Python ``random``;
with ``num_envs`` > 1 each env draws its own exploration coin.
"""
from __future__ import annotations

import csv
import math
import os
import random
from typing import Optional

import numpy as np
import torch

from . import _lib
from .engine import SwarmEngine, flatten_state_dict, glorot_init, unflatten_params
from .gcn import GCN
from .graph import Batch, Data, create_graph_from_observations


class SummaryWriter:
    """Minimal stand-in for torch.utils.tensorboard.SummaryWriter (not installed):
    keeps the scalars the reference logs ('Loss', 'Reward'; :136,174) in memory."""

    def __init__(self, *args, **kwargs):
        self.scalars = {}

    def add_scalar(self, tag, value, step):
        self.scalars.setdefault(tag, []).append((int(step), float(value)))

    def close(self):
        pass


class GraphReplayBuffer:
    """Ring of (graph, actions, rewards, next_graph) with the reference's push/sample/len.

    Standalone buffer for API users; stores node features on the device.  The
    fused trainer uses the engine's SoA replay ring instead (same semantics,
    one slot per tick holding every env's transition)."""

    def __init__(self, capacity: int):
        self.capacity = capacity
        self.buffer = []
        self.position = 0

    def push(self, graph_observation, actions, rewards, next_graph_observation):
        if len(self.buffer) < self.capacity:
            self.buffer.append(None)
        self.buffer[self.position] = (graph_observation, actions, rewards, next_graph_observation)
        self.position = (self.position + 1) % self.capacity

    def sample(self, batch_size: int):
        sample = random.sample(self.buffer, batch_size)
        obs = [s[0] for s in sample]
        acts = [s[1] for s in sample]
        rews = [s[2] for s in sample]
        nxt = [s[3] for s in sample]
        return Batch.from_data_list(obs), torch.cat(acts), torch.cat(rews), Batch.from_data_list(nxt)

    def __len__(self):
        return len(self.buffer)


class _EngineReplayView:
    """len() view of the engine's replay ring, in graphs."""

    def __init__(self, engine: SwarmEngine):
        self.engine = engine

    def __len__(self):
        return self.engine.replay_len()


def set_seed(seed: int):
    """train_gcn_dqn.py:233-239."""
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)


class DQNTrainer:
    def __init__(self, env, seed: int, models_path: str, stats_path: str, experiment: str, *,
                 batch_size: int = 32, update_target_every: int = 200, lr: float = 1e-3, gamma: float = 0.99,
                 replay_capacity: int = 1_000_000, use_graph: bool = True):
        self.env = env
        self.seed = seed
        self.models_path = models_path
        self.stats_path = stats_path
        self.experiment = experiment
        self.n_input = env.observation_space["agent0"].shape[0] + 1
        self.n_output = env.action_space["agent0"].n
        self.model = GCN(input_dim=self.n_input, hidden_dim=32, output_dim=self.n_output)
        init = glorot_init(torch.Generator().manual_seed(seed))
        self.model.load_state_dict(unflatten_params(init))
        self.target_model = GCN(input_dim=self.n_input, hidden_dim=32, output_dim=self.n_output)
        self.target_model.load_state_dict(self.model.state_dict())
        self.batch_size = batch_size
        self.update_target_every = update_target_every
        self.use_graph = use_graph
        scen = env.scenario
        self.engine = SwarmEngine(scenario=scen.SCENARIO_ID, n_agents=env.n_agents, n_envs=env.num_envs,
                                  seed=seed, params=init, batch=batch_size, gamma=gamma, lr=lr,
                                  update_target_every=update_target_every, replay_capacity=replay_capacity,
                                  shared_reset=True, random_oa=bool(getattr(scen, "random", False)))
        self.optimizer = SimpleAdamView(self.engine)
        self.replay_buffer = _EngineReplayView(self.engine)
        self.writer = SummaryWriter()
        self.episode_rewards = []
        self.episode_losses = []
        self.episode_obstacle_hits = []
        self.rewards_buffer = []
        self.obstacle_hits_buffer = []

    def create_graph_from_observations(self, observations) -> Data:
        return create_graph_from_observations(observations)

    def _sync_models(self):
        self.engine.flush()
        self.model.load_state_dict(unflatten_params(self.engine.params.detach().cpu()))
        self.target_model.load_state_dict(unflatten_params(self.engine.target.detach().cpu()))

    def train_step_dqn(self, batch_size, model=None, target_model=None, ticks=None, gamma=0.99,
                       update_target_every=10) -> float:
        """One TD update on the engine's replay (train_gcn_dqn.py:112-137)."""
        if len(self.replay_buffer) < batch_size:
            print("Not enough samples in the replay buffer")
            return 0
        eng = self.engine
        eng.hp.batch = batch_size
        eng.hp.gamma = gamma
        eng.hp.update_target_every = update_target_every
        if ticks is not None:   # the kernels sync when (ctrl.tick + 1) % every == 0
            eng.ctrl[0] = int(ticks) - 1
        eng.td_update()
        c = eng.read_ctrl()
        self._sync_models()
        self.writer.add_scalar("Loss", c["loss"], c["tick"])
        return c["loss"]

    def _episode_fn(self, max_steps: int):
        """One training tick plus the bookkeeping the reference does on the host every tick
        (train_gcn_dqn.py:174-177), kept on the device: the episode's reward and loss sums, and
        per tick the summed agent reward ('Reward', :174), the TD loss and whether an update
        ran ('Loss' is logged only by updates, :113-115,136).  The tick's slot in the per-tick
        buffers is fixed when the call is made, so a captured episode replays into the same
        slots; train_model reads them once per episode."""
        eng = self.engine
        n = self.env.n_agents
        calls = [0]

        def tick():
            i = calls[0] % max_steps
            calls[0] += 1
            eng.train_tick(full_out=False)
            self._acc_reward.add_(eng.reward[:, 0].mean() / n)
            self._acc_loss.add_(eng.ctrl.view(torch.float32)[5])
            self._tick_reward[i].copy_(eng.reward.sum(dim=1).mean())
            self._tick_loss[i].copy_(eng.ctrl.view(torch.float32)[5])
            self._tick_trained[i].copy_(eng.ctrl[7])
        return tick

    def train_model(self, config):
        eng = self.engine
        initial_epsilon = config["epsilon"]
        epsilon_decay = config["epsilon_decay"]
        min_epsilon = config["min_epsilon"]
        episodes = config["episodes"]
        max_steps = self.env.max_steps or 100
        epsilon = initial_epsilon
        self._acc_reward = torch.zeros((), device=eng.device)
        self._acc_loss = torch.zeros((), device=eng.device)
        self._tick_reward = torch.zeros(max_steps, device=eng.device)
        self._tick_loss = torch.zeros(max_steps, device=eng.device)
        self._tick_trained = torch.zeros(max_steps, dtype=torch.int32, device=eng.device)
        tick_fn = self._episode_fn(max_steps)
        ticks = 0
        graph = None
        for episode in range(episodes):
            eng.reset()
            eng.set_eps(epsilon)
            self._acc_reward.zero_()
            self._acc_loss.zero_()
            if self.use_graph and episode > 0:
                if graph is None:   # episode 0 ran eagerly (warm-up); capture one whole episode once
                    graph = eng.capture(max_steps, tick_fn)
                graph.replay()
            else:
                for _ in range(max_steps):
                    tick_fn()
            epsilon = max(min_epsilon, initial_epsilon * np.exp(-epsilon_decay * episode))
            average_loss = float(self._acc_loss.item()) / max_steps
            ep_reward = float(self._acc_reward.item())
            # the per-tick scalars of the episode, read once (train_gcn_dqn.py:136,174)
            rew_t, loss_t, tr_t = self._tick_reward.tolist(), self._tick_loss.tolist(), self._tick_trained.tolist()
            for i in range(max_steps):
                ticks += 1
                self.writer.add_scalar("Reward", rew_t[i], ticks)
                if tr_t[i]:
                    self.writer.add_scalar("Loss", loss_t[i], ticks)
            eng.check_handoffs()   # an overrun hand-off dropped TD graphs: fail loudly (one 4-byte read)
            if eng.peer is not None:
                eng.peer.check()   # an expired peer-exchange wait: the summed gradient is wrong
            self.episode_losses.append(average_loss)
            self.rewards_buffer.append(torch.tensor(ep_reward))
            if (episode + 1) % 10 == 0:
                self.episode_rewards.append(sum(self.rewards_buffer) / 10)
                self.rewards_buffer = []
            print(f"Episode {episode}, Loss: {average_loss}, Reward: {ep_reward * self.env.n_agents}, "
                  f"Epsilon: {epsilon}")
        print("Training completed")
        self._sync_models()
        os.makedirs(self.models_path, exist_ok=True)
        torch.save(self.model.state_dict(), f"{self.models_path}/experiment_{self.experiment}-seed_{self.seed}.pth")
        print("Model saved successfully!")
        self.save_metrics_to_csv()

    def save_metrics_to_csv(self):
        os.makedirs(self.stats_path, exist_ok=True)
        with open(f"{self.stats_path}/experiment_{self.experiment}-seed_{self.seed}.csv", mode="w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Episode", "Reward", "Loss"])
            for i in range(len(self.episode_losses)):
                if (i + 1) % 10 == 0:   # reference quirk: losses indexed with i // 10 (:231)
                    w.writerow([i, float(self.episode_rewards[i // 10]), self.episode_losses[i // 10]])


class SimpleAdamView:
    """Exposes the device Adam state the way code inspecting ``trainer.optimizer`` expects."""

    def __init__(self, engine: SwarmEngine):
        self.engine = engine

    def state_dict(self):
        e = self.engine
        return {"step": e.read_ctrl()["adam_step"], "exp_avg": e.adam_m.cpu(), "exp_avg_sq": e.adam_v.cpu(),
                "lr": e.hp.lr, "betas": (e.hp.beta1, e.hp.beta2), "eps": e.hp.eps}
