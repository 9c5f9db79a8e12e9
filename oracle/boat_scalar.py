"""SCALAR CPU ORACLE for one boat env — TEST / BASELINE INFRASTRUCTURE, NOT PRODUCT CODE.

Only ``tests/`` and ``bench.py``'s ``cpu_baseline`` leg (through
``tools/cpu_c1.py``) may import this module. The product path never does.

SURVEY.md §7.2's "scalar N=1 mode": the reference's ``BoatEnv`` for ONE env,
restated with Python floats and the ``math`` module, the way the reference
runs (one env per process, ``main.py:70-91``), without numpy's per-call cost on
1-element arrays. The step follows Nilau1998/SAC-Agent line by line:

* ``BoatEnv.step``           environment/boat_env.py:67-115
* ``BoatEnv.reset``          environment/boat_env.py:120-126
* ``Boat.__init__``          environment/boat_env.py:144-201 (``randint`` :147-150)
* ``Boat.run_model_step``    environment/boat_env.py:203-211
* ``eom_longitudinal``       environment/boat_env.py:213-239
* ``eom_transverse``         environment/boat_env.py:241-265
* ``eom_yawning``            environment/boat_env.py:267-281
* ``get_kinematics``         environment/boat_env.py:283-306
* ``return_state``           environment/boat_env.py:308-326
* ``Integrator``             environment/control_theory/control_blocks.py:5-36
* ``Wind``                   environment/wind.py:12-99 -- the reference materialises the
  per-episode wind tables at reset (``interp1d`` over 10 000 samples, min-max
  renormalisation); so does this class, with the spline basis of
  ``boat_oracle.spline_basis`` (numpy at reset, as the reference's scipy call),
  and the step indexes the table (``wind.py:20-24``)
* ``exponential_reward``     environment/reward_functions.py:42-57

Pinned against the reference-generated fixtures by tests/test_oracle_golden.py
(``test_scalar_oracle_matches_seeded_fixtures``).
"""
from __future__ import annotations

import math

import numpy as np

from boat_oracle import (OracleConfig, TERM_FUEL, TERM_GOAL, TERM_NONE, TERM_OOB, TERM_RUDDER,
                         TERM_TIMEOUT, TERM_TRUNC, spline_basis)

_PI = math.pi


class ScalarBoat:
    """One reference ``BoatEnv`` (with its own legacy RandomState): env with seed s
    reproduces ``np.random.seed(s); env = BoatEnv(cfg)``."""

    def __init__(self, cfg: OracleConfig, seed: int, max_episode_steps: int = 0):
        if cfg.experiment not in (1, 2, 3, 4, 5, 6):
            raise ValueError("Well someone tried to use an experiment that doesnt exist!")
        self.cfg = cfg
        self.rng = np.random.RandomState(int(seed))
        self.max_episode_steps = int(max_episode_steps)
        c = cfg
        # constant products of the reference expressions, kept in its order below
        self.oob = c.track_width + c.oob_offset                  # boat_env.py:200-201
        self.m_mx = c.boat_m + c.boat_m_x
        self.m_my = c.boat_m + c.boat_m_y
        self.i_iz = c.boat_I + c.boat_Iz
        self.counters = [0, 0, 0, 0, 0]
        self.ep_reward = 0.0
        self._new_boat()                                          # boat_env.py:15

    # ------------------------------------------------------------------ reset
    def _curve(self) -> np.ndarray:
        """wind.py:69-90: knots, the interp1d samples, min-max renormalisation."""
        c = self.cfg
        kv = self.rng.random_sample(c.fixed_points)              # wind.py:78
        v = spline_basis(c.L, c.fixed_points) @ kv               # wind.py:82-84
        if np.any((v < 0) | (v > 1)):                            # wind.py:87-89
            v = (v - v.min()) / (v.max() - v.min())
        return v

    def _new_boat(self) -> None:
        """Boat(config) (boat_env.py:144-201) and its Wind (wind.py:26-67)."""
        c = self.cfg
        hw = int(c.track_width * 0.8)
        self.start_y = int(self.rng.randint(-hw, hw))           # :147-150
        L = c.L
        e = c.experiment
        if e in (1, 2):
            vel = ang = None
        elif e == 3:
            vel = ang = None
        elif e == 4:
            vel = (self._curve() * c.max_velocity).tolist()
            ang = None
        elif e == 5:
            cur = self._curve()
            vel = None
            ang = ((np.where(cur <= 0.5 / 2, 0.0, 1.0) * np.pi) + np.pi / 2).tolist()  # wind.py:92-99
        else:
            vel = (self._curve() * c.max_velocity).tolist()      # wind.py:58-63, velocity first
            ang = (self._curve() * np.pi * 2).tolist()
        self.wind_v, self.wind_a = vel, ang
        self.wind_v0 = c.max_velocity if e in (3, 5) else 0.0
        self.wind_a0 = c.direction * (_PI / 180) if e in (3, 4) else 0.0
        self.L = L
        self.s_x = self.s_r = 0.0
        self.v_x = self.v_y = self.v_r = 0.0
        self.a_x = self.a_y = self.a_r = 0.0
        self.rudder = 0.0
        self.t = 0.0
        self.index = 0
        self.fuel = c.fuel
        self.s_y = float(self.start_y) if e == 2 else 0.0        # :166-169, primed at :198

    def reset(self) -> list:
        """boat_env.py:120-126."""
        self._new_boat()
        self.ep_reward = 0.0
        return self.observe()

    # ------------------------------------------------------------------ obs
    def observe(self) -> list:
        """Boat.return_state (boat_env.py:308-326)."""
        c = self.cfg
        return [(self.s_x - 0) / (c.goal_line - 0), (self.v_x - 0) / (5 - 0),
                (self.a_x - 0) / (0.025 - 0),
                (self.s_y - -c.track_width) / (c.track_width - -c.track_width),
                (self.v_y - 0) / (2 - 0), (self.a_y - 0) / (0.37 - 0),
                (self.s_r - 0) / (2 * _PI - 0), (self.v_r - 0) / (8.5e-3 - 0),
                (self.a_r - 0) / (1.4e-5 - 0),
                (self.rudder - -_PI / 3) / (_PI / 3 - -_PI / 3),
                (float(self.fuel) - 0) / (c.fuel - 0)]

    # ------------------------------------------------------------------ step
    def step(self, action: float):
        """BoatEnv.step (boat_env.py:67-115) -> (obs, reward, term). ``action`` enters
        the rudder as float64 of the f32 value."""
        c = self.cfg
        self.t = self.t + c.dt                                   # :69
        self.fuel = self.fuel - 1                                # :70
        if c.test_mode == 0:                                     # :72-73
            self.rudder = self.rudder + float(action) / 10
        first = self.index == 0
        i = self.index if self.index < self.L else self.L - 1
        wv = self.wind_v[i] if self.wind_v is not None else self.wind_v0
        wa = self.wind_a[i] if self.wind_a is not None else self.wind_a0
        wsign = (wv > 0) - (wv < 0)

        # eom_longitudinal :213-239
        v_x = self.v_x
        F_R = v_x * v_x * c.c_r_front * 0.5 * c.rho * c.boat_area_front
        J = v_x * (1 - c.wake_friction) / (20 * c.propeller_diameter)
        F_T = math.sin(J) * (20 * 20) * c.rho * c.propeller_diameter ** 4 * (1 - c.thrust_deduction)
        F_C = self.v_y * self.m_my * self.v_r
        F_W = (wv * wv * wsign * c.c_r_front * 0.5 * c.rho * c.boat_area_front) * math.cos(wa)
        self.a_x = (-F_R + F_T + F_C + F_W) / self.m_mx
        self.v_x = v_x = 3.0 if first else self.a_x * c.dt + v_x

        # eom_transverse :241-265 (the new v_x)
        v_y = self.v_y
        F_R = v_y * v_y * c.c_r_side * 0.5 * c.rho * c.boat_area_side * ((v_y > 0) - (v_y < 0))
        sin_rud = math.sin(self.rudder)
        F_RU = sin_rud * (v_x * v_x * c.c_r_front * 0.5 * c.rho * c.rudder_area)
        F_C = v_x * self.m_mx * self.v_r
        F_W = (wv * wv * wsign * c.c_r_side * 0.5 * c.rho * c.boat_area_side) * math.sin(wa)
        self.a_y = (-F_R + F_RU + F_C + F_W) / self.m_my
        self.v_y = v_y = 0.0 if first else self.a_y * c.dt + v_y

        # eom_yawning :267-281
        v_r = self.v_r
        M_hull = v_r * v_r * c.c_r_side * 0.5 * c.rho * c.boat_area_side * c.boat_l * 5 * ((v_r > 0) - (v_r < 0))
        M_rud = (v_x * v_x * c.c_r_side * 0.5 * c.rho * c.rudder_area * sin_rud * (c.boat_b / 2)
                 * ((v_x > 0) - (v_x < 0)))
        self.a_r = (-M_hull + M_rud) / self.i_iz
        self.v_r = v_r = 0.0 if first else self.a_r * c.dt + v_r

        # get_kinematics :283-306
        v = math.sqrt(v_x * v_x + v_y * v_y)
        drift = math.atan2(v_x, v_y)
        self.s_r = v_r * c.dt + self.s_r
        direction = drift - self.s_r
        self.s_x = (math.sin(direction) * v) * c.dt + self.s_x
        self.s_y = (math.cos(direction) * v) * c.dt + self.s_y
        self.index += 1                                          # :211

        obs = self.observe()                                     # :77
        W = c.track_width                                        # reward_functions.py:42-57
        ay = abs(self.s_y)
        reward = 0 - (ay / W) / (1 + math.exp((-c.y_a / c.y_b) * (ay - (W * 0.2))))

        # termination chain :84-105
        if self.s_x >= c.goal_line:
            term = TERM_GOAL
            reward = reward + 1000
        elif abs(self.s_y) > self.oob or self.s_x < 0:
            term = TERM_OOB
        elif self.fuel < 0:
            term = TERM_FUEL
        elif c.t_max <= self.t:
            term = TERM_TIMEOUT
        elif self.rudder > _PI / 3 or self.rudder < -_PI / 3:
            term = TERM_RUDDER
        else:
            term = TERM_NONE
        if self.rudder > _PI / 4 or self.rudder < -_PI / 4:    # :107-111
            reward = reward - abs(self.rudder) * 100
        if abs(self.s_r) > _PI / 2:
            reward = reward - 1
        self.ep_reward = self.ep_reward + reward                 # :113
        if term != TERM_NONE:
            self.counters[term - 1] += 1                         # info-dict key order
        elif self.max_episode_steps > 0 and self.index >= self.max_episode_steps:
            term = TERM_TRUNC
        return obs, reward, term


__all__ = ["ScalarBoat", "TERM_FUEL", "TERM_GOAL", "TERM_NONE", "TERM_OOB", "TERM_RUDDER",
           "TERM_TIMEOUT", "TERM_TRUNC"]
