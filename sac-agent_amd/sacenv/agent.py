"""Batched SAC agent over a device replay buffer.

The reference trains one env at a time (main.py:70-114): ``choose_action``
copies one obs row to the device and the action back (continuous_agent.py:57-61),
``env.step`` runs on the CPU, ``remember`` stores into a numpy buffer. Here the
actor acts on all N observations at once ([N, 11] -> [N, 1]), the env steps in
one kernel and ``DeviceReplayBuffer`` appends the N transitions in one launch;
nothing crosses to the host.

``VecSAC.learn`` restates ``ContinuousAgent.learn`` (continuous_agent.py:96-154)
operation for operation, on the networks of networks/networks.py:14-133
(256-256 MLPs, tanh-squashed Normal policy with log-std in [-5, 2]) and the
agent section of configs/original_config.yaml. Two hooks make it checkable
against the reference (tests/test_gpu_parity.py, ``sac_learn.npz``):

* ``VecSAC(..., init_seed=s)`` builds the five networks on the CPU under
  ``torch.manual_seed(s)`` in the reference constructor's order (actor,
  critic 1, critic 2, value, target value; continuous_agent.py:19-51), so the
  initial weights are the reference agent's for the same seed;
* ``learn(batch=..., noise=...)`` takes the sampled batch and the standard
  normal draws of the policy's ``sample()`` / ``rsample()``
  (networks.py:58-61) explicitly.

The dense layers are torch (hipBLASLt) here; they are a different roofline
(MFMA) and outside this engine's tier.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F


@dataclass(frozen=True)
class AgentConfig:
    """configs/original_config.yaml:12-21 (agent section)."""
    lr_alpha: float = 0.005       # learning_rate_alpha (actor)
    lr_beta: float = 0.0003       # learning_rate_beta (critics, value)
    gamma: float = 0.99
    tau: float = 0.005            # tvn_parameter_modulation_tau
    max_size: int = 1_000_000
    layer1_size: int = 256
    layer2_size: int = 256
    batch_size: int = 1024
    reward_scale: float = 10

    @classmethod
    def from_any(cls, cfg=None) -> "AgentConfig":
        if cfg is None:
            return cls()
        if isinstance(cfg, cls):
            return cfg
        a = cfg.get("agent", cfg) if isinstance(cfg, dict) else getattr(cfg, "agent", cfg)
        get = (lambda k, d: a.get(k, d)) if isinstance(a, dict) else (lambda k, d: getattr(a, k, d))
        base = cls()
        return cls(lr_alpha=float(get("learning_rate_alpha", base.lr_alpha)),
                   lr_beta=float(get("learning_rate_beta", base.lr_beta)),
                   gamma=float(get("gamma", base.gamma)),
                   tau=float(get("tvn_parameter_modulation_tau", base.tau)),
                   max_size=int(get("max_size", base.max_size)),
                   layer1_size=int(get("layer1_size", base.layer1_size)),
                   layer2_size=int(get("layer2_size", base.layer2_size)),
                   batch_size=int(get("batch_size", base.batch_size)),
                   reward_scale=float(get("reward_scale", base.reward_scale)))


class Actor(nn.Module):
    """networks.py:14-70 ActorNetwork (layer order fc1, fc2, mean, std)."""

    def __init__(self, obs_dim=11, n_actions=1, max_action=1.0, h1=256, h2=256):
        super().__init__()
        self.fc1, self.fc2 = nn.Linear(obs_dim, h1), nn.Linear(h1, h2)
        self.mean, self.std = nn.Linear(h2, n_actions), nn.Linear(h2, n_actions)
        self.max_action, self.reparam_noise = float(max_action), 1e-6

    def sample_normal(self, state, reparameterize=True, eps=None):
        """networks.py:47-70; ``eps`` = the standard normal draws (else drawn here)."""
        x = F.relu(self.fc2(F.relu(self.fc1(state))))
        mean, std = self.mean(x), self.std(x)
        log_std = -5 + 0.5 * (2 - (-5)) * (torch.tanh(std) + 1)   # LOG_STD_MIN/MAX (:50-56)
        std = log_std.exp()
        normal = torch.distributions.Normal(mean, std)
        if eps is None:
            actions = normal.rsample() if reparameterize else normal.sample()
        elif reparameterize:
            actions = mean + eps * std
        else:
            with torch.no_grad():
                actions = mean + eps * std
        action = torch.tanh(actions) * self.max_action
        log_probs = normal.log_prob(actions)
        log_probs = log_probs - torch.log(1 - action.pow(2) + self.reparam_noise)
        return action, log_probs.sum(1, keepdim=True)


class Critic(nn.Module):
    """networks.py:73-104 CriticNetwork."""

    def __init__(self, obs_dim=11, n_actions=1, h1=256, h2=256):
        super().__init__()
        self.fc1, self.fc2, self.q = nn.Linear(obs_dim + n_actions, h1), nn.Linear(h1, h2), nn.Linear(h2, 1)

    def forward(self, state, action):
        return self.q(F.relu(self.fc2(F.relu(self.fc1(torch.cat([state, action], 1))))))


class Value(nn.Module):
    """networks.py:107-133 ValueNetwork."""

    def __init__(self, obs_dim=11, h1=256, h2=256):
        super().__init__()
        self.fc1, self.fc2, self.v = nn.Linear(obs_dim, h1), nn.Linear(h1, h2), nn.Linear(h2, 1)

    def forward(self, state):
        return self.v(F.relu(self.fc2(F.relu(self.fc1(state)))))


class VecSAC:
    """ContinuousAgent (continuous_agent.py:9-154) with a device buffer and batched acting."""

    NETS = ("actor", "critic_1", "critic_2", "value", "target_value")

    def __init__(self, device, config=None, *, obs_dim: int = 11, n_actions: int = 1,
                 max_action: float = 1.0, init_seed: int | None = None, buffer_seed: int = 0,
                 with_memory: bool = True):
        cfg = self.cfg = AgentConfig.from_any(config)
        h1, h2 = cfg.layer1_size, cfg.layer2_size
        build = lambda: (Actor(obs_dim, n_actions, max_action, h1, h2), Critic(obs_dim, n_actions, h1, h2),  # noqa: E731
                         Critic(obs_dim, n_actions, h1, h2), Value(obs_dim, h1, h2), Value(obs_dim, h1, h2))
        if init_seed is not None:
            with torch.random.fork_rng(devices=[]):
                torch.manual_seed(int(init_seed))
                nets = build()
        else:
            nets = build()
        self.actor, self.critic_1, self.critic_2, self.value, self.target_value = (n.to(device) for n in nets)
        self.device = torch.device(device)
        self.opt_actor = torch.optim.Adam(self.actor.parameters(), lr=cfg.lr_alpha)
        self.opt_c1 = torch.optim.Adam(self.critic_1.parameters(), lr=cfg.lr_beta)
        self.opt_c2 = torch.optim.Adam(self.critic_2.parameters(), lr=cfg.lr_beta)
        self.opt_value = torch.optim.Adam(self.value.parameters(), lr=cfg.lr_beta)
        self.update_network_parameters(tau=1.0)                          # :53
        self.memory = None
        if with_memory:
            from .replay import DeviceReplayBuffer
            self.memory = DeviceReplayBuffer(cfg.max_size, (obs_dim,), n_actions, device=device,
                                             seed=buffer_seed)

    @torch.no_grad()
    def choose_action(self, obs, eps=None):
        """[N, obs_dim] -> [N, n_actions] actions (continuous_agent.py:57-61), no host copy."""
        a, _ = self.actor.sample_normal(obs, reparameterize=False, eps=eps)
        return a

    @torch.no_grad()
    def update_network_parameters(self, tau=None):
        """continuous_agent.py:63-77: target <- tau * value + (1 - tau) * target."""
        tau = self.cfg.tau if tau is None else tau
        for tp, p in zip(self.target_value.parameters(), self.value.parameters()):
            tp.copy_(tau * p.clone() + (1 - tau) * tp.clone())

    def learn(self, batch=None, noise=None):
        """continuous_agent.py:96-154. ``batch`` = (state, action, reward, new_state, done)
        (else sampled from the device buffer, buffer.py:24-35); ``noise`` = (eps of the
        sample() draw, eps of the rsample() draw), each [B, n_actions].
        Returns (value_loss, actor_loss, critic_1_loss, critic_2_loss) or None."""
        if batch is None:
            if self.memory is None or self.memory.mem_cntr < self.cfg.batch_size:
                return None
            state, action, reward, state_, done, _ = self.memory.sample(self.cfg.batch_size)
        else:
            state, action, reward, state_, done = batch
        dev = self.device
        reward = torch.as_tensor(reward, device=dev).to(torch.float32)
        done = torch.as_tensor(done, device=dev).to(torch.bool)
        state_ = torch.as_tensor(state_, device=dev).to(torch.float32)
        state = torch.as_tensor(state, device=dev).to(torch.float32)
        action = torch.as_tensor(action, device=dev).to(torch.float32)
        e1, e2 = (None, None) if noise is None else (torch.as_tensor(n, device=dev) for n in noise)

        value = self.value(state).view(-1)
        value_ = self.target_value(state_).view(-1)
        value_ = torch.where(done, torch.zeros_like(value_), value_)    # value_[done] = 0.0

        actions, log_probs = self.actor.sample_normal(state, reparameterize=False, eps=e1)
        log_probs = log_probs.view(-1)
        critic_value = torch.min(self.critic_1(state, actions), self.critic_2(state, actions)).view(-1)

        self.opt_value.zero_grad()
        value_target = critic_value - log_probs
        value_loss = 0.5 * F.mse_loss(value, value_target)
        value_loss.backward(retain_graph=True)
        self.opt_value.step()

        actions, log_probs = self.actor.sample_normal(state, reparameterize=True, eps=e2)
        log_probs = log_probs.view(-1)
        critic_value = torch.min(self.critic_1(state, actions), self.critic_2(state, actions)).view(-1)
        actor_loss = torch.mean(log_probs - critic_value)
        self.opt_actor.zero_grad()
        actor_loss.backward(retain_graph=True)
        self.opt_actor.step()

        self.opt_c1.zero_grad()
        self.opt_c2.zero_grad()
        q_hat = self.cfg.reward_scale * reward + self.cfg.gamma * value_.detach()
        critic_1_loss = 0.5 * F.mse_loss(self.critic_1(state, action).view(-1), q_hat)
        critic_2_loss = 0.5 * F.mse_loss(self.critic_2(state, action).view(-1), q_hat)
        (critic_1_loss + critic_2_loss).backward()
        self.opt_c1.step()
        self.opt_c2.step()
        self.update_network_parameters()
        return tuple(x.detach() for x in (value_loss, actor_loss, critic_1_loss, critic_2_loss))

    def state_dicts(self) -> dict:
        return {n: getattr(self, n).state_dict() for n in self.NETS}

    def optimizer_state(self) -> dict:
        return {n: o.state_dict() for n, o in zip(self.NETS[:4], (self.opt_actor, self.opt_c1,
                                                                   self.opt_c2, self.opt_value))}

    def load_optimizer_state(self, state: dict) -> None:
        for n, o in zip(self.NETS[:4], (self.opt_actor, self.opt_c1, self.opt_c2, self.opt_value)):
            o.load_state_dict(state[n])

    def save_models(self, experiment_dir: str, optimizer: bool = False) -> None:
        """ContinuousAgent.save_models (continuous_agent.py:79-84): see ``save_models``."""
        save_models(self, experiment_dir, optimizer)

    def load_models(self, experiment_dir: str, optimizer: bool = False) -> None:
        """ContinuousAgent.load_models (continuous_agent.py:86-91): see ``load_models``."""
        load_models(self, experiment_dir, optimizer)


# checkpoint file of each net: the reference's network names (continuous_agent.py:19-52),
# under <experiment_dir>/checkpoints/ (networks/base_network.py:10-11)
CHECKPOINT_NAMES = {"actor": "actor_network", "critic_1": "critic_network_1",
                    "critic_2": "critic_network_2", "value": "value_network",
                    "target_value": "target_value_network"}
OPTIMIZER_FILE = "sac_optimizer"  # not in the reference: the Adam states, for exact resumes


def save_models(agent, experiment_dir: str, optimizer: bool = False) -> None:
    """Each net's ``state_dict`` to ``<experiment_dir>/checkpoints/<name>`` with
    ``torch.save``, as BaseNetwork.save_checkpoint (networks/base_network.py:13-14)
    writes it: the reference's ``load_checkpoint`` reads these files unchanged.
    Tensors are saved as CPU copies (a parameter that views a larger device buffer
    would otherwise carry the whole buffer). ``optimizer`` also writes the Adam
    states (``OPTIMIZER_FILE``; the reference keeps none), so a resumed agent
    continues bit for bit."""
    import os
    d = os.path.join(experiment_dir, "checkpoints")
    os.makedirs(d, exist_ok=True)
    for n in agent.NETS:
        sd = {k: v.detach().cpu().clone() for k, v in getattr(agent, n).state_dict().items()}
        torch.save(sd, os.path.join(d, CHECKPOINT_NAMES[n]))
    if optimizer:
        torch.save(agent.optimizer_state(), os.path.join(d, OPTIMIZER_FILE))


def load_models(agent, experiment_dir: str, optimizer: bool = False) -> None:
    """BaseNetwork.load_checkpoint (networks/base_network.py:16-17) for every net;
    ``weights_only`` loads (the files hold tensors only)."""
    import os
    d = os.path.join(experiment_dir, "checkpoints")
    for n in agent.NETS:
        sd = torch.load(os.path.join(d, CHECKPOINT_NAMES[n]), map_location="cpu", weights_only=True)
        getattr(agent, n).load_state_dict(sd)
    if optimizer:
        agent.load_optimizer_state(torch.load(os.path.join(d, OPTIMIZER_FILE), map_location="cpu",
                                              weights_only=True))
    if hasattr(agent, "sync"):
        agent.sync()


__all__ = ["AgentConfig", "Actor", "Critic", "Value", "VecSAC", "save_models", "load_models",
           "CHECKPOINT_NAMES"]
