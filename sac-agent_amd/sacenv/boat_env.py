"""Drop-in ``BoatEnv`` (one env, numpy in/out) over the HIP engine.

Mirrors the surface the reference's callers touch:
``BoatEnv(config, experiment)`` (main.py:43), ``observation_space.shape``
(main.py:50), ``reset()`` (main.py:72), the 4-tuple ``step(action)``
(main.py:81), the single aliased ``info`` dict with cumulative counters
(boat_env.py:24-32, main.py:83,110,132-133), ``env.boat.rudder_angle`` and
``env.action`` (main.py:94-96), ``return_all_data`` / ``experiment_dir`` /
``boat.wind.wind_velocity|wind_angle`` (postprocessing/recorder.py:14-48),
and a gym ``Box`` action space (agent/base_agent.py:9-17).

RNG: by default the env draws from numpy's GLOBAL legacy stream, exactly
like the reference (``np.random.randint`` boat_env.py:147, ``np.random.sample``
wind.py:78): before each Boat construction the global MT19937 state is
uploaded to the GPU, the reset kernel consumes the draws there, and the
advanced state is written back with ``np.random.set_state``. Interleaving
with other ``np.random`` users (the replay buffer, buffer.py:27) is
therefore identical to the reference. Pass ``rng=<int>`` for a private
stream instead.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from .config import BoatConfig, observation_bounds
from .spaces import Box
from .vec_env import VecBoatEnv


class _WindView:
    """``Boat.wind`` (wind.py:5-24): tables evaluated on the GPU on demand."""

    def __init__(self, env: "BoatEnv"):
        self._env = env
        self._cache = None

    def _tables(self):
        if self._cache is None or self._cache[0] != self._env._episode:
            L = self._env._cfg.wind_len
            v, a = self._env._vec.wind_eval(np.zeros(L, np.int32), np.arange(L, dtype=np.int32))
            torch.cuda.synchronize(self._env._vec.device)
            self._cache = (self._env._episode, v.cpu().numpy(), a.cpu().numpy())
        return self._cache

    @property
    def wind_velocity(self) -> np.ndarray:
        return self._tables()[1]

    @property
    def wind_angle(self) -> np.ndarray:
        return self._tables()[2]

    def get_wind(self, index: int) -> np.ndarray:
        return np.array([self.wind_velocity[index], self.wind_angle[index]])


class _BoatView:
    """Read-only view of ``Boat`` attributes (boat_env.py:143-201) from device state."""

    n = 20  # boat_env.py:178

    def __init__(self, env: "BoatEnv"):
        self._env = env
        self.wind = _WindView(env)
        cfg = env._cfg
        self.dt, self.t_max = cfg.dt, cfg.t_max
        self.out_of_bounds = cfg.track_width + cfg.boat_out_of_bounds_offset

    def _get(self, name):
        return self._env._host_state()[name]

    s_x = property(lambda self: float(self._get("s_x")))
    s_y = property(lambda self: float(self._get("s_y")))
    s_r = property(lambda self: float(self._get("s_r")))
    v_x = property(lambda self: float(self._get("v_x")))
    v_y = property(lambda self: float(self._get("v_y")))
    v_r = property(lambda self: float(self._get("v_r")))
    a_x = property(lambda self: float(self._get("a_x")))
    a_y = property(lambda self: float(self._get("a_y")))
    a_r = property(lambda self: float(self._get("a_r")))
    rudder_angle = property(lambda self: float(self._get("rudder")))
    t = property(lambda self: float(self._get("t")))
    fuel = property(lambda self: int(self._get("fuel")))
    index = property(lambda self: int(self._get("index")))
    s_y_start = property(lambda self: int(self._get("start_y")))


class BoatEnv:
    """One boat env with the reference ``BoatEnv`` surface (boat_env.py:9-140)."""

    def __init__(self, config=None, experiment=None, *, device=None, rng="global"):
        self.config = config
        self._cfg = BoatConfig.from_any(config)
        self.experiment_dir = getattr(experiment, "experiment_dir", None)
        self.action = [0]
        self.reward = 0
        self._global_rng = rng == "global"
        seed = 0 if self._global_rng else int(rng)
        # the arena's own init draw is replaced by _new_boat() below
        self._vec = VecBoatEnv(self._cfg, 1, seed=seed, device=device, autoreset=False,
                               record_accel=True, record_reward64=True)
        self._episode = 0
        self._hs = None
        self.info = {"termination": "", "reached_goal": 0, "out_of_bounds": 0,
                     "out_of_fuel": 0, "rudder_broken": 0, "timeout": 0,
                     "episode_reward": 0}
        self.action_space = Box(low=-1, high=1, dtype=np.float32)
        self.low_state, self.high_state = observation_bounds()
        self.observation_space = Box(low=self.low_state, high=self.high_state, dtype=np.float32)
        # one pinned host round trip per step: the action in, then one packed copy
        # out (obs f32 x 11 | reward f64 | term u8) instead of three blocking reads
        dev = self._vec.device
        self._act_host = torch.empty(1, dtype=torch.float32).pin_memory()
        self._act_dev = torch.empty(1, dtype=torch.float32, device=dev)
        self._out_dev = torch.empty(53, dtype=torch.uint8, device=dev)
        self._out_host = torch.empty(53, dtype=torch.uint8).pin_memory()
        self._new_boat()                         # boat_env.py:15
        self.boat = _BoatView(self)

    # -------------------------------------------------------------- RNG mirror
    def _rng_in(self):
        if not self._global_rng:
            return None
        st = np.random.get_state(legacy=True)
        key = np.asarray(st[1], dtype=np.uint32)
        self._vec.mt_key[0].copy_(torch.from_numpy(key.view(np.int32)))
        self._vec.mt_pos[0] = int(st[2])
        return st

    def _rng_out(self, st):
        if st is None:
            return
        torch.cuda.synchronize(self._vec.device)
        key = self._vec.mt_key[0].cpu().numpy().view(np.uint32).copy()
        pos = int(self._vec.mt_pos[0].item()) & 0xFFFF   # (bit 16: the refill's pre-twisted block)
        np.random.set_state((st[0], key, pos, st[3], st[4]))

    def _new_boat(self):
        st = self._rng_in()
        self._vec.reset()
        self._rng_out(st)
        self._episode += 1
        self._hs = None

    def _host_state(self) -> dict:
        if self._hs is None:
            self._hs = {k: v[0] for k, v in self._vec.state_dict().items()}
        return self._hs

    # -------------------------------------------------------------- gym API
    def step(self, action):
        """boat_env.py:67-115 -> (state, reward, done, info)."""
        self.action = action
        v = self._vec
        self._act_host[0] = float(np.asarray(action, dtype=np.float32).reshape(-1)[0])
        self._act_dev.copy_(self._act_host, non_blocking=True)
        v.step_async(self._act_dev)
        out = self._out_dev
        out[:44].copy_(v.obs[0].view(torch.uint8))
        out[44:52].copy_(v.reward64[:1].view(torch.uint8))
        out[52:].copy_(v.term[:1])
        self._out_host.copy_(out, non_blocking=True)
        torch.cuda.current_stream(v.device).synchronize()
        self._hs = None
        h = self._out_host.numpy()
        obs = h[:44].view(np.float32).astype(np.float64)
        self.reward = float(h[44:52].view(np.float64)[0])
        code = int(h[52])
        done = code != _lib.TERM_NONE
        if done and code <= _lib.TERM_TIMEOUT:
            name = _lib.TERM_NAMES[code]
            self.info["termination"] = name
            self.info[name] += 1
        self.info["episode_reward"] += self.reward
        self.state = obs
        return obs, self.reward, done, self.info

    def render(self):
        pass

    def reset(self):
        """boat_env.py:120-126."""
        self._new_boat()
        self.info["episode_reward"] = 0
        torch.cuda.synchronize(self._vec.device)
        self.state = self._vec.obs[0].cpu().numpy().astype(np.float64)
        return self.state

    def return_all_data(self) -> dict:
        """boat_env.py:128-140 (the Recorder's CSV row)."""
        b = self.boat
        return {"boat_position_x": b.s_x, "boat_position_y": b.s_y,
                "boat_velocity_x": b.v_x, "boat_velocity_y": b.v_y,
                "boat_angle": b.s_r, "action_rudder": self.action[0],
                "reward": self.reward, "rudder_angle": b.rudder_angle, "n": b.n}
