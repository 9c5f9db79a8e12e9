"""Config handling: the reference's YAML layout -> SacenvBoatParams.

The reference reads its constants from ``configs/original_config.yaml`` via
``utils/config_reader.py:6-14`` (YAML -> DotMap, attribute access). This
module accepts the same shapes: a path to such a YAML, a nested dict, or any
object with attribute access (a DotMap), and builds the C params struct.
Defaults are the reference's ``original_config.yaml`` values (lines 2-65).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, fields, replace

import numpy as np

from . import _lib


@dataclass(frozen=True)
class BoatConfig:
    # base_settings (original_config.yaml:2-9)
    experiment: int = 5
    test_mode: int = 0
    dt: float = 0.25
    t_max: float = 2500
    # boat_env (:27-30)
    track_width: float = 800
    boat_out_of_bounds_offset: float = 0
    goal_line: float = 3900
    # boat (:33-61)
    fuel: int = 15000
    boat_m: float = 600
    boat_m_x: float = 50
    boat_m_y: float = 100
    boat_I: float = 6_000_000
    boat_Iz: float = 10
    propeller_diameter: float = 1
    wake_friction: float = 0.3
    c_r_front: float = 0.31
    c_r_side: float = 2
    thrust_deduction: float = 0.3
    rho: float = 1
    boat_area_front: float = 20
    boat_area_side: float = 90
    boat_l: float = 15
    boat_b: float = 6
    rudder_area: float = 10
    # wind (:63-66)
    fixed_points: int = 8
    max_velocity: float = 0.5
    direction: float = 90

    _SECTIONS = {
        "base_settings": ("experiment", "test_mode", "dt", "t_max"),
        "boat_env": ("track_width", "boat_out_of_bounds_offset", "goal_line"),
        "boat": ("fuel", "boat_m", "boat_m_x", "boat_m_y", "boat_I", "boat_Iz",
                 "propeller_diameter", "wake_friction", "c_r_front", "c_r_side",
                 "thrust_deduction", "rho", "boat_area_front", "boat_area_side", "boat_l",
                 "boat_b", "rudder_area"),
        "wind": ("fixed_points", "max_velocity", "direction"),
    }

    @property
    def wind_len(self) -> int:
        return int(self.t_max / self.dt)            # wind.py:14-15

    @classmethod
    def from_any(cls, cfg=None, **overrides) -> "BoatConfig":
        """From None (defaults), a BoatConfig, a YAML path, a nested dict or a DotMap."""
        if cfg is None:
            base = cls()
        elif isinstance(cfg, BoatConfig):
            base = cfg
        else:
            if isinstance(cfg, str):
                import yaml
                with open(cfg) as f:
                    cfg = yaml.safe_load(f)
            kw = {}
            for sect, keys in cls._SECTIONS.items():
                src = _get(cfg, sect)
                if src is None:
                    continue
                for k in keys:
                    v = _get(src, k)
                    if v is not None:
                        kw[k] = v
            base = cls(**kw)
        return replace(base, **overrides) if overrides else base

    def validate(self) -> None:
        if int(self.experiment) not in (1, 2, 3, 4, 5, 6):   # wind.py:65-67
            raise ValueError("Well someone tried to use an experiment that doesnt exist!")
        if int(self.experiment) in (4, 5, 6) and int(self.fixed_points) < 4:  # wind.py:73-75
            raise ValueError("Please select at least 4 fixed_points in your config. "
                             "The interpolation doesn't work otherwise!")
        if int(self.fixed_points) > _lib.MAX_KNOTS:
            raise ValueError(f"fixed_points > {_lib.MAX_KNOTS} is not supported")
        if int(self.track_width * 0.8) < 1:
            raise ValueError("low >= high in np.random.randint: int(0.8*track_width) must be >= 1")
        if self.wind_len < 2:
            raise ValueError("t_max/dt must give at least 2 wind samples")


def _get(obj, key):
    if isinstance(obj, dict):
        return obj.get(key)
    return getattr(obj, key, None)


def t_from_index(dt: float) -> bool:
    """Mirror of the kernel's rule: ``t += dt`` is exact (t == index * dt) when
    dt's significand has at most 22 bits; the kernel then keeps no t in HBM."""
    bits = np.array([dt], dtype=np.float64).view(np.uint64)[0]
    return int(bits) & ((1 << 30) - 1) == 0


def spline_g(n: int) -> np.ndarray:
    """G with (second derivative / 6) = G @ knot_values for the not-a-knot cubic.

    The interpolant scipy's ``interp1d(kind='cubic')`` builds (wind.py:82-84)
    on n uniformly spaced knots, in the knot coordinate s = x / h:
    interior rows m[j-1] + 4 m[j] + m[j+1] = 6 (y[j-1] - 2 y[j] + y[j+1]),
    end rows m[0] - 2 m[1] + m[2] = 0 and m[n-3] - 2 m[n-2] + m[n-1] = 0
    (third derivative continuous at the first and last interior knot).
    """
    A = np.zeros((n, n))
    R = np.zeros((n, n))
    A[0, 0:3] = (1.0, -2.0, 1.0)
    A[n - 1, n - 3:n] = (1.0, -2.0, 1.0)
    for j in range(1, n - 1):
        A[j, j - 1:j + 2] = (1.0, 4.0, 1.0)
        R[j, j - 1:j + 2] = (6.0, -12.0, 6.0)
    return np.linalg.solve(A, R) / 6.0


def make_params(cfg: BoatConfig, n_envs: int, *, max_episode_steps: int = 0,
                autoreset: bool = True, n_helpers: int = 8192, out_flags: int = 0,
                use_wind_table: bool = False) -> _lib.BoatParams:
    cfg.validate()
    p = _lib.BoatParams()
    p.n_envs = int(n_envs)
    p.experiment = int(cfg.experiment)
    p.test_mode = int(cfg.test_mode)
    p.wind_len = cfg.wind_len
    p.n_knots = int(cfg.fixed_points)
    p.fuel0 = int(cfg.fuel)
    p.start_y_half = int(cfg.track_width * 0.8)     # boat_env.py:147-150
    p.max_episode_steps = int(max_episode_steps)
    p.autoreset = 1 if autoreset else 0
    p.n_helpers = int(n_helpers)
    p.out_flags = int(out_flags)
    p.use_wind_table = 1 if use_wind_table else 0
    p.dt = float(cfg.dt)
    p.t_max = float(cfg.t_max)
    p.goal_line = float(cfg.goal_line)
    p.oob_limit = float(cfg.track_width + cfg.boat_out_of_bounds_offset)  # :200-201
    p.track_width = float(cfg.track_width)
    for f in ("c_r_front", "c_r_side", "rho", "boat_area_front", "boat_area_side", "boat_l",
              "boat_b", "rudder_area"):
        setattr(p, f, float(getattr(cfg, f)))
    # sums/differences the reference forms from config values (one IEEE op each)
    p.m_plus_mx = float(cfg.boat_m + cfg.boat_m_x)              # boat_env.py:239
    p.m_plus_my = float(cfg.boat_m + cfg.boat_m_y)              # :230, :265
    p.i_plus_iz = float(cfg.boat_I + cfg.boat_Iz)               # :281
    p.one_minus_wf = float(1 - cfg.wake_friction)               # :221
    p.one_minus_td = float(1 - cfg.thrust_deduction)            # :227
    n, D = 20, cfg.propeller_diameter                           # :178
    p.n_rpm = float(n)
    p.n_times_d = float(n * D)                                  # :224
    p.n_squared = float(np.square(n))                           # :226
    p.d_pow4 = float(np.power(D, 4))                            # :226
    p.max_velocity = float(cfg.max_velocity)
    p.wind_dir_rad = float(cfg.direction) * (math.pi / 180)     # wind.py:370
    p.reward_k = (-0.03) / 3.4                                  # (-y_a/y_b), boat_env.py:21-22
    p.reward_center = float(cfg.track_width) * 0.2              # reward_functions.py:53
    p.knot_step = (cfg.fixed_points - 1) / (cfg.wind_len - 1)
    p.knot_inv = (cfg.wind_len - 1) / (cfg.fixed_points - 1)
    return p


def observation_bounds():
    """low_state / high_state of boat_env.py:49-60 (float32)."""
    low = np.array([0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1], dtype=np.float32)
    high = np.array([1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0], dtype=np.float32)
    return low, high


def first_obs_template(cfg: BoatConfig) -> np.ndarray:
    """Boat.return_state of a fresh Boat (boat_env.py:152-198, :308-326) as the step
    kernel writes it (f32): every state value 0 but fuel = fuel0; entry 3 is
    (s_y + W) / 2W = 0.5 at s_y = 0 (experiment 2 starts at its start y: the
    pooled transition row carries that entry as obs3_next)."""
    rud0 = np.float32((0.0 + np.pi / 3) * (1.0 / (np.pi / 3 - (-np.pi / 3))))
    with np.errstate(invalid="ignore", divide="ignore"):
        fuel = np.float64(cfg.fuel) / np.float64(cfg.fuel) if cfg.fuel else np.float64(np.nan)
    t = np.zeros(11, np.float32)
    t[3], t[9], t[10] = 0.5, rud0, np.float32(fuel)
    return t


__all__ = ["BoatConfig", "make_params", "spline_g", "observation_bounds", "t_from_index",
           "first_obs_template"]
_ = fields  # keep dataclasses import explicit for readers
