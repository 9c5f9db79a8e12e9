"""Vectorised toy integrator envs and the mixed batch (one launch).

The reference's toy scripts, environment/toy_parachute.py:7-41 and
environment/toy_car.py:5-33, are open-loop loops over control_blocks.py:5-36
Integrators with no Gym surface. Here each becomes an env whose ``step`` is
one iteration of that loop for every env on the GPU:

* parachute: obs [s, v], done when the script would stop (s < 0: the
  script's break, term 1; or t > t_max after ``t += dt``: term 5);
* car: obs [s_x, s_y], done at t > t_max (term 5);
* reward 0; ``max_episode_steps`` truncates (term 6); auto-reset restarts
  from the scripts' initial variables.

``MixedBatch`` steps a ``VecBoatEnv`` and toy envs in ONE kernel launch with
heterogeneous workgroups (BASELINE.json configs[4]).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib
from .spaces import Box

TOY_RECORD_BYTES = 14  # obs f32x2 | reward f32 | done u8 | term u8


@dataclass(frozen=True)
class ParachuteConfig:
    """Constants of toy_parachute.py:11-21 (Integrator dt: control_blocks.py:7)."""
    h0: float = 3000
    h1: float = 1500
    area_closed: float = 0.5     # A_s
    area_open: float = 25        # A_FS
    mass: float = 85
    c_w: float = 1.3
    rho: float = 1.2             # p
    g: float = 9.81
    dt: float = 0.01
    t_max: float = 500
    integ_dt: float = 0.1


@dataclass(frozen=True)
class CarConfig:
    """Constants of toy_car.py:8-20, :24 (Integrator dt: control_blocks.py:7)."""
    accel: float = 10            # car_max_a, the a-integrator's input
    v_max: float = 10            # Integrator(upper_limit=10)
    dangle: float = 0.01
    dt: float = 0.1
    t_max: float = 500
    integ_dt: float = 0.1


def make_toy_params(kind: int, cfg, n_envs: int, *, autoreset: bool = True,
                    max_episode_steps: int = 0) -> _lib.ToyParams:
    p = _lib.ToyParams()
    p.n_envs = int(n_envs)
    p.kind = int(kind)
    p.autoreset = 1 if autoreset else 0
    p.max_episode_steps = int(max_episode_steps)
    p.dt, p.t_max, p.integ_dt = float(cfg.dt), float(cfg.t_max), float(cfg.integ_dt)
    if kind == _lib.TOY_PARACHUTE:
        for f in ("h0", "h1", "area_closed", "area_open", "mass", "c_w", "rho", "g"):
            setattr(p, f, float(getattr(cfg, f)))
    elif kind == _lib.TOY_CAR:
        p.car_accel, p.car_v_max, p.car_dangle = float(cfg.accel), float(cfg.v_max), float(cfg.dangle)
    else:
        raise ValueError(f"unknown toy kind {kind}")
    return p


class VecToyEnv:
    """``num_envs`` copies of one toy script's loop, resident on one GPU."""

    obs_dim = 2

    def __init__(self, kind: int, config=None, num_envs: int = 1, *, device=None,
                 max_episode_steps: int = 0, autoreset: bool = True):
        self.lib = _lib.load()
        self.kind = int(kind)
        if config is None:
            config = ParachuteConfig() if self.kind == _lib.TOY_PARACHUTE else CarConfig()
        self.cfg = config
        self.num_envs = N = int(num_envs)
        if N <= 0:
            raise ValueError("num_envs must be positive")
        self.device = torch.device(device if device is not None else "cuda")
        if self.device.type != "cuda":
            raise RuntimeError("VecToyEnv runs on a GPU (HIP); no CPU path")
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.autoreset = bool(autoreset)
        self.params = make_toy_params(self.kind, config, N, autoreset=autoreset,
                                      max_episode_steps=max_episode_steps)
        self._pp = C.byref(self.params)
        self.layout = L = _lib.toy_layout(self.params)
        self.n_pad = NP = int(L.n_pad)
        self.arena = torch.zeros(int(L.total_bytes), dtype=torch.uint8, device=self.device)

        def view(off, dtype, *shape):
            esz = torch.empty((), dtype=dtype).element_size()
            cnt = int(np.prod(shape))
            return self.arena[off: off + cnt * esz].view(dtype).view(*shape)

        self.state = view(L.state, torch.float64, 5, NP)[:, :N]
        self.count = view(L.count, torch.int32, NP)[:N]
        self.counters = view(L.counters, torch.int32, 3, NP)[:, :N]
        self.record = self.arena[L.record: L.record + TOY_RECORD_BYTES * NP]
        self.obs = view(L.obs, torch.float32, NP, 2)[:N]
        self.reward = view(L.reward, torch.float32, NP)[:N]
        self.done = view(L.done, torch.uint8, NP)[:N]
        self.term = view(L.term, torch.uint8, NP)[:N]
        self.final_obs = view(L.final_obs, torch.float32, NP, 2)[:N]
        self.final_obs_bytes = self.arena[L.final_obs: L.final_obs + 8 * NP]
        # gym-style metadata: open-loop envs take no action
        self.action_space = Box(low=0, high=0, shape=(0,), dtype=np.float32)
        self.observation_space = Box(low=-np.inf, high=np.inf, shape=(2,), dtype=np.float32)
        _lib.check(self.lib.sacenv_toy_init(self._pp, self.arena.data_ptr(), self.stream))

    @property
    def stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    def reset(self, env_ids=None) -> torch.Tensor:
        if env_ids is None:
            _lib.check(self.lib.sacenv_toy_reset(self._pp, self.arena.data_ptr(), None, 0, self.stream))
        else:
            ids = torch.as_tensor(env_ids, dtype=torch.int32, device=self.device).contiguous()
            if ids.numel():
                _lib.check(self.lib.sacenv_toy_reset(self._pp, self.arena.data_ptr(), ids.data_ptr(),
                                                     ids.numel(), self.stream))
                self._keep = ids
        return self.obs

    def step_async(self, actions=None) -> None:
        _lib.check(self.lib.sacenv_toy_step(self._pp, self.arena.data_ptr(), self.stream))

    def step(self, actions=None):
        """One loop iteration for every env -> (obs, reward, done, info) device views."""
        self.step_async()
        return self.obs, self.reward, self.done, {"term": self.term, "final_obs": self.final_obs,
                                                  "counters": self.counters}


class ParachuteEnv(VecToyEnv):
    def __init__(self, config=None, num_envs: int = 1, **kw):
        super().__init__(_lib.TOY_PARACHUTE, config, num_envs, **kw)


class CarEnv(VecToyEnv):
    def __init__(self, config=None, num_envs: int = 1, **kw):
        super().__init__(_lib.TOY_CAR, config, num_envs, **kw)


class MixedBatch:
    """A boat env and up to two toy envs stepped by ONE heterogeneous launch."""

    def __init__(self, boat=None, toys=()):
        toys = list(toys)
        if len(toys) > 2:
            raise ValueError("at most two toy envs per mixed launch")
        if boat is None and not toys:
            raise ValueError("empty mixed batch")
        devs = {e.device for e in ([boat] if boat is not None else []) + toys}
        if len(devs) != 1:
            raise ValueError("all envs of a mixed batch must be on one device")
        self.boat, self.toys = boat, toys
        self.lib = _lib.load()
        self._tp = (_lib.ToyParams * max(1, len(toys)))(*[t.params for t in toys])
        self._ta = (C.c_void_p * max(1, len(toys)))(*[t.arena.data_ptr() for t in toys])

    @property
    def num_envs(self) -> int:
        return (self.boat.num_envs if self.boat is not None else 0) + sum(t.num_envs for t in self.toys)

    def step_async(self, boat_actions=None, trans_row=None) -> None:
        """One heterogeneous launch; ``trans_row`` (boat only): the boat's pooled
        transition row as ``VecBoatEnv.step_pooled_async`` writes it."""
        b = self.boat
        stream = (b if b is not None else self.toys[0]).stream
        if b is not None:
            a = torch.as_tensor(boat_actions, device=b.device)
            if a.dtype != torch.float32:
                a = a.to(torch.float32)
            a = a.reshape(b.num_envs).contiguous()
            b.check_actions(a)
            self._keep = a
        if trans_row is not None:
            if b is None:
                raise ValueError("a transition row needs the boat env")
            if (trans_row.dtype != torch.uint8 or trans_row.device != b.device or not trans_row.is_contiguous()
                    or trans_row.numel() != _lib.trans_bytes(b.params.experiment) * b.n_pad):
                raise ValueError("trans_row must be a contiguous uint8 device tensor of "
                                 "trans_bytes(experiment) * n_pad bytes")
            _lib.check(self.lib.sacenv_mixed_step_pooled(
                b._pp, b.arena.data_ptr(), a.data_ptr(), self._tp, self._ta, len(self.toys),
                trans_row.data_ptr(), stream))
        else:
            _lib.check(self.lib.sacenv_mixed_step(
                b._pp if b is not None else None, b.arena.data_ptr() if b is not None else None,
                a.data_ptr() if b is not None else None, self._tp, self._ta, len(self.toys), stream))
        if b is not None:
            b._after_step()

    def segment_async(self, boat_actions=None, n_steps: int | None = None) -> None:
        """``n_steps`` steps of the whole batch in ONE persistent launch
        (``sacenv_mixed_segment``): the same results as ``n_steps`` ``step_async``
        calls, bit for bit. ``boat_actions``: a [K >= n_steps, N] f32 device tensor
        with contiguous rows (row k drives step k; rows may be strided)."""
        b = self.boat
        stream = (b if b is not None else self.toys[0]).stream
        a = None
        if b is not None:
            a = boat_actions
            K = int(a.shape[0]) if n_steps is None else int(n_steps)
            if (not isinstance(a, torch.Tensor) or a.dtype != torch.float32 or a.device != b.device
                    or a.dim() != 2 or a.shape[1] != b.num_envs or a.stride(1) != 1 or a.shape[0] < K):
                raise ValueError(f"boat_actions must be a float32 [>= {K}, {b.num_envs}] device tensor "
                                 "with contiguous rows")
            if b.autoreset and K > _lib.REFILL_PERIOD:
                raise ValueError(f"a segment of more than {_lib.REFILL_PERIOD} steps in autoreset mode")
            if b.autoreset and b.auto_refill and b._since_refill + K > _lib.REFILL_PERIOD:
                b.refill()
            self._keep = a
        else:
            K = int(n_steps)
        _lib.check(self.lib.sacenv_mixed_segment(
            b._pp if b is not None else None, b.arena.data_ptr() if b is not None else None,
            a.data_ptr() if a is not None else None, int(a.stride(0)) if a is not None else 0, K,
            self._tp, self._ta, len(self.toys), stream))
        if b is not None and b.autoreset:
            b._since_refill += K


__all__ = ["ParachuteConfig", "CarConfig", "VecToyEnv", "ParachuteEnv", "CarEnv", "MixedBatch",
           "make_toy_params"]
