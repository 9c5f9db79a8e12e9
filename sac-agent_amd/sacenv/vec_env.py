"""VecBoatEnv: N boat envs per GPU behind the reference's Gym surface.

Batched counterpart of ``BoatEnv`` (environment/boat_env.py:9-140). Every
env is an independent reference ``BoatEnv`` with its own numpy-legacy RNG
stream: env ``e`` seeded with ``s`` behaves exactly like
``np.random.seed(s); env = BoatEnv(cfg)`` in the reference — the constructor
builds one Boat (boat_env.py:15) and every ``reset`` another (:121).

All compute runs in libsacenv.so (gfx950 HIP); tensors here are device
memory plumbing. ``step`` enqueues one kernel on the current torch stream and
never synchronises.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _lib
from .config import BoatConfig, make_params, observation_bounds, spline_g
from .spaces import Box

RECORD_BYTES = 50  # packed per-env record: obs f32x11 | reward f32 | done u8 | term u8


def _ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


class VecBoatEnv:
    """``num_envs`` boat envs resident on one GPU.

    Parameters
    ----------
    config : reference-style config (YAML path, dict, DotMap) or BoatConfig.
    num_envs : envs on this device.
    seed : base seed; env ``e`` gets ``seeds[e] = (seed + env_id_offset + e) mod 2**32``
        unless ``seeds`` is given explicitly.
    max_episode_steps : >0 truncates episodes (term code 6) after that many steps.
    autoreset : reset ended envs inside ``step`` (gym vector-env semantics:
        the returned obs row is the new episode's first obs, the terminal obs
        is in ``info['final_obs']``).
    env_id_offset : global id of this rank's first env (multi-GPU sharding).
    record_knots : also keep the raw drawn knot values (parity tests).
    """

    def __init__(self, config=None, num_envs: int = 1, *, seed: int = 0, seeds=None,
                 device=None, max_episode_steps: int = 0, autoreset: bool = True,
                 env_id_offset: int = 0, record_knots: bool = False, wind_table=None,
                 _skip_init_reset: bool = False):
        self.lib = _lib.load()
        self.cfg = BoatConfig.from_any(config)
        self.num_envs = N = int(num_envs)
        if N <= 0:
            raise ValueError("num_envs must be positive")
        self.device = torch.device(device if device is not None else "cuda")
        if self.device.type != "cuda":
            raise RuntimeError("VecBoatEnv runs on a GPU (HIP); no CPU path")
        self.env_id_offset = int(env_id_offset)
        self.params = make_params(self.cfg, N, max_episode_steps=max_episode_steps,
                                  autoreset=autoreset)
        dev, f64, i32 = self.device, torch.float64, torch.int32
        nk = int(self.cfg.fixed_points)

        def z(dtype, *shape):
            return torch.zeros(*shape, dtype=dtype, device=dev)

        # carried state, SoA
        self.s_x, self.s_y, self.s_r = z(f64, N), z(f64, N), z(f64, N)
        self.v_x, self.v_y, self.v_r = z(f64, N), z(f64, N), z(f64, N)
        self.rudder, self.t, self.ep_reward = z(f64, N), z(f64, N), z(f64, N)
        self.index, self.start_y = z(i32, N), z(i32, N)
        self.wind_y = z(f64, 2, nk, N)
        self.wind_m = z(f64, 2, nk, N)
        self.knots_raw = z(f64, 2, nk, N) if record_knots else None
        self.mt_key = z(i32, N, _lib.MT_N)
        self.mt_pos = z(i32, N)
        self.counters = z(i32, _lib.N_COUNTERS, N)
        self._spline_g = torch.as_tensor(spline_g(nk), dtype=f64, device=dev).contiguous()
        self.params.spline_g = self._spline_g.data_ptr()
        self._wind_table = None
        if wind_table is not None:
            wt = torch.as_tensor(np.asarray(wind_table, np.float64).reshape(2, -1), device=dev)
            if wt.shape[1] != self.cfg.wind_len:
                raise ValueError("wind_table must be [2, int(t_max/dt)]")
            self._wind_table = wt.contiguous()
            self.params.wind_table = self._wind_table.data_ptr()

        # outputs: one packed record buffer (the all-gather payload), plus extras
        self.record = z(torch.uint8, N * RECORD_BYTES)
        self.obs = self.record[: 44 * N].view(torch.float32).view(N, _lib.OBS_DIM)
        self.reward = self.record[44 * N: 48 * N].view(torch.float32)
        self.done = self.record[48 * N: 49 * N]
        self.term = self.record[49 * N: 50 * N]
        self.final_obs = z(torch.float32, N, _lib.OBS_DIM)
        self.final_ep_reward = z(f64, N)
        self.accel = z(f64, 3, N)
        self.reward64 = z(f64, N)

        self.state = _lib.BoatState(
            s_x=_ptr(self.s_x), s_y=_ptr(self.s_y), s_r=_ptr(self.s_r),
            v_x=_ptr(self.v_x), v_y=_ptr(self.v_y), v_r=_ptr(self.v_r),
            rudder=_ptr(self.rudder), t=_ptr(self.t), ep_reward=_ptr(self.ep_reward),
            index=_ptr(self.index), start_y=_ptr(self.start_y),
            wind_y=_ptr(self.wind_y), wind_m=_ptr(self.wind_m), knots_raw=_ptr(self.knots_raw),
            mt_key=_ptr(self.mt_key), mt_pos=_ptr(self.mt_pos), counters=_ptr(self.counters))
        self.out = _lib.BoatStepOut(
            obs=_ptr(self.obs), reward=_ptr(self.reward), done=_ptr(self.done),
            term=_ptr(self.term), final_obs=_ptr(self.final_obs),
            final_ep_reward=_ptr(self.final_ep_reward), accel=_ptr(self.accel),
            reward64=_ptr(self.reward64))
        self._pp, self._ps, self._po = C.byref(self.params), C.byref(self.state), C.byref(self.out)

        # Gym surface (boat_env.py:37-65)
        self.action_space = Box(low=-1, high=1, dtype=np.float32)
        low, high = observation_bounds()
        self.observation_space = Box(low=low, high=high, dtype=np.float32)

        if seeds is None:
            gid = np.arange(N, dtype=np.uint64) + np.uint64(self.env_id_offset)
            seeds = (np.uint64(seed) + gid) & np.uint64(0xFFFFFFFF)
        seeds = np.asarray(seeds, dtype=np.uint64)
        if seeds.shape != (N,):
            raise ValueError("seeds must have one entry per env")
        if np.any(seeds > 0xFFFFFFFF):
            raise ValueError("Seed must be between 0 and 2**32 - 1")
        self.seeds = seeds
        self.seed(seeds)
        if not _skip_init_reset:
            self._reset_all()   # BoatEnv.__init__ builds a Boat (boat_env.py:15)

    # ------------------------------------------------------------------ plumbing
    @property
    def stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    def seed(self, seeds) -> None:
        """np.random.seed(seeds[e]) for every env (legacy MT19937 init)."""
        s = torch.from_numpy(np.asarray(seeds, np.uint64).astype(np.uint32).view(np.int32))
        self._seeds_dev = s.to(self.device)
        _lib.check(self.lib.sacenv_boat_seed(self._pp, self._ps, self._seeds_dev.data_ptr(),
                                             self.stream))

    def _reset_all(self) -> None:
        _lib.check(self.lib.sacenv_boat_reset(self._pp, self._ps, None, 0,
                                              self.obs.data_ptr(), self.stream))

    # ------------------------------------------------------------------ gym API
    def reset(self, env_ids=None) -> torch.Tensor:
        """BoatEnv.reset for all envs, or for ``env_ids`` (boat_env.py:120-126)."""
        if env_ids is None:
            self._reset_all()
        else:
            ids = torch.as_tensor(env_ids, dtype=torch.int32, device=self.device).contiguous()
            if ids.numel():
                _lib.check(self.lib.sacenv_boat_reset(self._pp, self._ps, ids.data_ptr(),
                                                      ids.numel(), self.obs.data_ptr(),
                                                      self.stream))
        return self.obs

    def reset_explicit(self, env_ids, start_y, knots=None) -> torch.Tensor:
        """Reset with caller-supplied draws (replaying recorded episodes)."""
        ids = torch.as_tensor(env_ids, dtype=torch.int32, device=self.device).contiguous()
        sy = torch.as_tensor(start_y, dtype=torch.int32, device=self.device).contiguous()
        kn = None
        if knots is not None:
            kn = torch.as_tensor(knots, dtype=torch.float64, device=self.device).contiguous()
        _lib.check(self.lib.sacenv_boat_reset_explicit(
            self._pp, self._ps, ids.data_ptr(), ids.numel(), sy.data_ptr(),
            None if kn is None else kn.data_ptr(), self.obs.data_ptr(), self.stream))
        self._keep = (ids, sy, kn)  # alive until the stream has consumed them
        return self.obs

    def step_async(self, actions: torch.Tensor) -> None:
        """Enqueue one step; ``actions`` is a contiguous f32 device tensor [N] or [N, 1]."""
        _lib.check(self.lib.sacenv_boat_step(self._pp, self._ps, actions.data_ptr(),
                                             self._po, self.stream))

    def step(self, actions):
        """BoatEnv.step for all envs (boat_env.py:67-115).

        Returns ``(obs, reward, done, info)`` as device tensors that alias the
        env's output buffers (overwritten by the next step; clone to keep).
        ``info`` holds ``term`` (SACENV_TERM_* codes; 1..5 in the order of the
        reference info-dict keys), ``final_obs`` and ``final_ep_reward``
        (valid where done) and the cumulative ``counters``.
        """
        a = torch.as_tensor(actions, device=self.device)
        if a.dtype != torch.float32:
            a = a.to(torch.float32)
        a = a.reshape(self.num_envs).contiguous()
        self._last_action = a
        self.step_async(a)
        info = {"term": self.term, "final_obs": self.final_obs,
                "final_ep_reward": self.final_ep_reward, "counters": self.counters}
        return self.obs, self.reward, self.done, info

    def wind_eval(self, env_ids, idx):
        """Wind.get_wind(index) for (env, index) pairs -> (velocity, angle) f64."""
        ids = torch.as_tensor(env_ids, dtype=torch.int32, device=self.device).contiguous()
        ix = torch.as_tensor(idx, dtype=torch.int32, device=self.device).contiguous()
        if ids.shape != ix.shape:
            raise ValueError("env_ids and idx must have the same shape")
        v = torch.empty(ids.shape, dtype=torch.float64, device=self.device)
        a = torch.empty_like(v)
        _lib.check(self.lib.sacenv_boat_wind_eval(self._pp, self._ps, ids.data_ptr(),
                                                  ix.data_ptr(), ids.numel(), v.data_ptr(),
                                                  a.data_ptr(), self.stream))
        return v, a

    def state_dict(self) -> dict:
        """Host copy of the carried state (parity tests / checkpoints)."""
        torch.cuda.synchronize(self.device)
        d = {k: getattr(self, k).cpu().numpy() for k in
             ("s_x", "s_y", "s_r", "v_x", "v_y", "v_r", "rudder", "t", "ep_reward",
              "index", "start_y")}
        d["fuel"] = int(self.cfg.fuel) - d["index"].astype(np.int64)
        d["a_x"], d["a_y"], d["a_r"] = self.accel.cpu().numpy()
        return d

    @property
    def counters_dict(self) -> dict:
        c = self.counters.cpu().numpy().astype(np.int64)
        return {name: c[k] for k, name in enumerate(_lib.TERM_NAMES[1:6])}
