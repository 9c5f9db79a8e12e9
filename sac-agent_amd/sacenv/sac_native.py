"""The SAC agent on the fp32 MFMA kernels of sacenv_sac.hip.

``NativeSAC`` has ``VecSAC``'s surface (sacenv/agent.py: ``choose_action``,
``learn(batch, noise)``, ``update_network_parameters``, ``state_dicts``, the five
``nn.Module`` attributes, a ``DeviceReplayBuffer`` as ``memory``), but
``choose_action`` is one ``sacenv_sac_act`` launch and ``learn`` is one
``sacenv_sac_learn`` call (four launches): ContinuousAgent.learn
(agent/continuous_agent.py:96-154) with all five networks, the four Adam
states (torch.optim.Adam, continuous_agent.py / networks.py:29-31 defaults)
and the target soft update in one device weights buffer.

The modules' parameters are views of that buffer, so ``state_dict()`` and the
reference's checkpoint format see the live weights; a host write into them
must be followed by ``sync()`` (the kernels keep a transposed copy of each
256x256 layer). Initial weights are the reference agent's for the same
``init_seed`` (the nets are built as VecSAC builds them).

There is no CPU path: without libsacenv.so or a GPU this class raises.
"""
from __future__ import annotations

import ctypes as C

import torch
import torch.nn as nn

from . import _lib
from .agent import AgentConfig, VecSAC, load_models, save_models

# torch parameter names per net, in the C layout's tensor order (w1, b1, w2, b2, head 0, head 1)
_TENSORS = {
    "actor": ("fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias", "mean.weight", "mean.bias",
              "std.weight", "std.bias"),
    "critic": ("fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias", "q.weight", "q.bias"),
    "value": ("fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias", "v.weight", "v.bias"),
}
_SHAPE = {"actor": 0, "critic_1": 1, "critic_2": 1, "value": 2, "target_value": 2}
_KIND = {"actor": "actor", "critic_1": "critic", "critic_2": "critic", "value": "value",
         "target_value": "value"}


def _set_param(module: nn.Module, dotted: str, t: torch.Tensor) -> None:
    mod_name, pname = dotted.split(".")
    setattr(getattr(module, mod_name), pname, nn.Parameter(t, requires_grad=False))


class NativeSAC:
    """ContinuousAgent (continuous_agent.py:9-154) on libsacenv's SAC kernels."""

    NETS = VecSAC.NETS

    def __init__(self, device, config=None, *, obs_dim: int = 11, n_actions: int = 1,
                 max_action: float = 1.0, init_seed: int | None = None, buffer_seed: int = 0,
                 with_memory: bool = True, adam_eps: float = 1e-8):
        cfg = self.cfg = AgentConfig.from_any(config)
        if cfg.layer1_size != _lib.SAC_HIDDEN or cfg.layer2_size != _lib.SAC_HIDDEN:
            raise ValueError(f"the SAC kernels are built for {_lib.SAC_HIDDEN}-wide layers")
        if n_actions != 1:
            raise ValueError("the SAC kernels take one action dimension (the boat's)")
        dev = torch.device(device)
        if dev.type != "cuda":
            raise _lib.SacenvError("NativeSAC runs on the GPU only (libsacenv SAC kernels)")
        self.device = torch.device("cuda", dev.index if dev.index is not None else torch.cuda.current_device())
        self.params = _lib.SacParams(
            obs_dim=obs_dim, n_actions=1, hidden=_lib.SAC_HIDDEN, batch=cfg.batch_size,
            max_action=float(max_action), gamma=cfg.gamma, tau=cfg.tau,
            reward_scale=cfg.reward_scale, lr_actor=cfg.lr_alpha, lr_critic=cfg.lr_beta,
            adam_beta1=0.9, adam_beta2=0.999, adam_eps=float(adam_eps))
        L = self.layout = _lib.sac_layout(self.params)
        self.weights = torch.zeros(L.total_floats, dtype=torch.float32, device=self.device)
        self.scratch = torch.empty(L.scratch_bytes // 4, dtype=torch.float32, device=self.device)
        self.losses = torch.zeros(4, dtype=torch.float32, device=self.device)
        # the reference's initial weights (VecSAC builds them under init_seed on the CPU)
        ref = VecSAC("cpu", cfg, obs_dim=obs_dim, n_actions=1, max_action=max_action,
                     init_seed=init_seed, with_memory=False)
        for i, name in enumerate(self.NETS):
            m = getattr(ref, name)
            for pname, view in self._views(self.weights, L.net[i], name).items():
                src = m.state_dict()[pname]
                view.copy_(src.reshape(view.shape))
                _set_param(m, pname, view)
            setattr(self, name, m.to(self.device))
        self.adam_step = 0
        self.sync()
        self.memory = None
        if with_memory:
            from .replay import DeviceReplayBuffer
            self.memory = DeviceReplayBuffer(cfg.max_size, (obs_dim,), n_actions, device=self.device,
                                             seed=buffer_seed)

    def _views(self, buf: torch.Tensor, base: int, name: str) -> dict:
        L, s, kind = self.layout, _SHAPE[name], _KIND[name]
        ins = {"actor": self.params.obs_dim, "critic": self.params.obs_dim + 1,
               "value": self.params.obs_dim}[kind]
        H = _lib.SAC_HIDDEN
        shapes = ((H, ins), (H,), (H, H), (H,), (1, H), (1,), (1, H), (1,))
        out = {}
        for k, pname in enumerate(_TENSORS[kind]):
            off = base + L.tensor[s][k]
            n = 1
            for d in shapes[k]:
                n *= d
            out[pname] = buf[off: off + n].view(*shapes[k])
        return out

    def adam_state(self, name: str) -> dict:
        """exp_avg / exp_avg_sq views of an optimised net (as torch.optim.Adam's state)."""
        i = self.NETS.index(name)
        if i > 3:
            raise KeyError(name)
        return {"exp_avg": self._views(self.weights, self.layout.adam_m[i], name),
                "exp_avg_sq": self._views(self.weights, self.layout.adam_v[i], name)}

    def _stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def sync(self) -> None:
        """Refresh the kernels' transposed 256x256 layers after a host write to the weights."""
        _lib.check(_lib.load().sacenv_sac_sync(C.byref(self.params), self.weights.data_ptr(),
                                               self._stream()))

    @torch.no_grad()
    def update_network_parameters(self, tau=None):
        """continuous_agent.py:63-77 (learn() applies it in-kernel)."""
        tau = self.cfg.tau if tau is None else tau
        for tp, p in zip(self.target_value.parameters(), self.value.parameters()):
            tp.copy_(tau * p.clone() + (1 - tau) * tp.clone())
        # the target's fc2.weight has a kernel copy in fragment order (role_critic_loss
        # reads it): refresh it, or the next learn() would use the stale target
        self.sync()

    def _f32(self, x, n=None):
        t = torch.as_tensor(x, device=self.device).to(torch.float32).contiguous()
        if n is not None and t.numel() != n:
            raise ValueError(f"expected {n} values, got {tuple(t.shape)}")
        return t

    @torch.no_grad()
    def choose_action(self, obs, eps=None):
        """[N, obs_dim] -> [N, 1] (continuous_agent.py:57-61): one kernel launch."""
        obs = self._f32(obs)
        if obs.dim() != 2 or obs.shape[1] != self.params.obs_dim:
            raise ValueError(f"obs must be [N, {self.params.obs_dim}], got {tuple(obs.shape)}")
        n = obs.shape[0]
        eps = torch.randn(n, device=self.device) if eps is None else self._f32(eps, n)
        out = torch.empty((n, 1), dtype=torch.float32, device=self.device)
        _lib.check(_lib.load().sacenv_sac_act(C.byref(self.params), self.weights.data_ptr(), obs.data_ptr(),
                                              n, eps.data_ptr(), out.data_ptr(), None, self._stream()))
        return out

    @torch.no_grad()
    def choose_action_handoff(self, obs, eps, out, *, obs_ready, obs_want: int, act_ready, act_value: int,
                              status=None) -> None:
        """``choose_action`` as the producer of a closed loop with ``VecBoatEnv.segment_async``
        (``sacenv_sac_act_handoff``): the 64 rows of block b (owner wave b's envs) are read once
        ``obs_ready[b] >= obs_want`` and ``act_ready[b] = act_value`` is published once their
        actions in ``out`` (f32 [N], device) are visible. Enqueued on the current stream."""
        n = obs.shape[0]
        if obs.dtype != torch.float32 or not obs.is_contiguous() or obs.shape[1] != self.params.obs_dim:
            raise ValueError(f"obs must be a contiguous float32 [N, {self.params.obs_dim}] tensor")
        for name, t, cnt in (("eps", eps, n), ("out", out, n)):
            if t.dtype != torch.float32 or not t.is_contiguous() or t.numel() != cnt or t.device != self.device:
                raise ValueError(f"{name} must be a contiguous float32 device tensor of {cnt} values")
        _lib.check(_lib.load().sacenv_sac_act_handoff(
            C.byref(self.params), self.weights.data_ptr(), obs.data_ptr(), n, eps.data_ptr(), out.data_ptr(),
            obs_ready.data_ptr(), int(obs_want), act_ready.data_ptr(), int(act_value),
            None if status is None else status.data_ptr(), self._stream()))

    @torch.no_grad()
    def learn(self, batch=None, noise=None, *, losses: bool = True):
        """continuous_agent.py:96-154 as VecSAC.learn; returns the four losses (device scalars,
        independent tensors), or with ``losses=False`` the agent's own f32 [4] loss buffer (no
        copy launch: the next learn() rewrites it). None while the buffer holds < batch rows."""
        B, D = self.cfg.batch_size, self.params.obs_dim
        if batch is None:
            if self.memory is None or self.memory.mem_cntr < B:
                return None
            state, action, reward, state_, done, _ = self.memory.sample(B, as_bool=False)
        else:
            state, action, reward, state_, done = batch
        state = self._f32(state, B * D)
        state_ = self._f32(state_, B * D)
        action = self._f32(action, B)
        reward = torch.as_tensor(reward, device=self.device).to(torch.float64).contiguous()
        done = torch.as_tensor(done, device=self.device).to(torch.uint8).contiguous()
        if reward.numel() != B or done.numel() != B:
            raise ValueError("reward and done must hold one value per batch row")
        if noise is None:
            e1, e2 = torch.randn(B, device=self.device), torch.randn(B, device=self.device)
        else:
            e1, e2 = self._f32(noise[0], B), self._f32(noise[1], B)
        step = self.adam_step + 1  # committed only once the call is accepted
        _lib.check(_lib.load().sacenv_sac_learn(
            C.byref(self.params), self.weights.data_ptr(), self.scratch.data_ptr(), state.data_ptr(),
            action.data_ptr(), reward.data_ptr(), state_.data_ptr(), done.data_ptr(), e1.data_ptr(),
            e2.data_ptr(), step, self.losses.data_ptr(), self._stream()))
        self.adam_step = step
        if not losses:
            return self.losses
        # independent tensors (as VecSAC.learn returns): the next learn() rewrites self.losses
        return tuple(self.losses.clone().unbind(0))

    def state_dicts(self) -> dict:
        return {n: getattr(self, n).state_dict() for n in self.NETS}

    def optimizer_state(self) -> dict:
        """The Adam moments of the four optimised nets and the step count (CPU copies)."""
        out = {"step": torch.tensor(self.adam_step, dtype=torch.int64)}
        for n in self.NETS[:4]:
            for which, views in self.adam_state(n).items():
                out.update({f"{n}.{which}.{k}": v.detach().cpu().clone() for k, v in views.items()})
        return out

    def load_optimizer_state(self, state: dict) -> None:
        for n in self.NETS[:4]:
            for which, views in self.adam_state(n).items():
                for k, v in views.items():
                    v.copy_(state[f"{n}.{which}.{k}"].reshape(v.shape))
        self.adam_step = int(state["step"])

    def save_models(self, experiment_dir: str, optimizer: bool = False) -> None:
        """ContinuousAgent.save_models (continuous_agent.py:79-84), the reference's files."""
        save_models(self, experiment_dir, optimizer)

    def load_models(self, experiment_dir: str, optimizer: bool = False) -> None:
        """ContinuousAgent.load_models (continuous_agent.py:86-91): the parameters are views
        of the weights buffer, so load_state_dict writes it in place; then sync()."""
        load_models(self, experiment_dir, optimizer)


__all__ = ["NativeSAC"]
