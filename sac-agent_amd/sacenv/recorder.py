"""Episode traces for a sampled subset of envs: postprocessing/recorder.py:7-56.

The reference's ``Recorder`` writes, for its single env, the following files
under ``<experiment_dir>/episodes/``:

* ``episode_<k>_data.csv``: one row of ``BoatEnv.return_all_data()``
  (boat_env.py:128-140) per step, written BEFORE the step (main.py:79).
* ``info.csv``: the info dict after each episode (main.py:100).
* ``wind.csv``: the first episode's wind tables (main.py:101).

All three are ';'-separated. ``VecRecorder`` keeps that format for K chosen envs of
a ``VecBoatEnv``, one reference-style ``episodes/`` folder per env
(``<experiment_dir>/episodes/env_<id>/``), so the reference's replay and rendering
tools can read any of them.

The step loop stays on the device:

* ``record()`` gathers the K rows into a device buffer;
* ``after_step()`` gathers the K done / term / episode-reward values;
* rows reach the host only in ``flush()``, every ``flush_steps`` steps or on
  ``close()``.
"""
from __future__ import annotations

import csv
import os

import numpy as np
import torch

from . import _lib

COLUMNS = ("boat_position_x", "boat_position_y", "boat_velocity_x", "boat_velocity_y",
           "boat_angle", "action_rudder", "reward", "rudder_angle", "n")
INFO_KEYS = ("termination", "reached_goal", "out_of_bounds", "out_of_fuel", "rudder_broken",
             "timeout", "episode_reward")          # boat_env.py:24-32 (dict order)
N_RPM = 20                                          # Boat.n (boat_env.py:178)


def _fmt(x: float) -> str:
    return repr(float(x))


class VecRecorder:
    def __init__(self, env, env_ids, experiment_dir: str, flush_steps: int = 512):
        self.env = env
        self.ids = torch.as_tensor(env_ids, dtype=torch.long, device=env.device)
        self.ids_host = [int(i) for i in self.ids.cpu()]
        self.K = len(self.ids_host)
        self.flush_steps = int(flush_steps)
        self.dirs = [os.path.join(experiment_dir, "episodes", f"env_{i}") for i in self.ids_host]
        for d in self.dirs:
            os.makedirs(d, exist_ok=True)
        self.episode = [0] * self.K
        self._rows, self._events = [], []
        # BoatEnv.__init__: action = [0], reward = 0 (boat_env.py:13-14)
        self._last_action = torch.zeros(self.K, dtype=torch.float64, device=env.device)
        self._last_reward = torch.zeros(self.K, dtype=torch.float64, device=env.device)
        self._wind_done = [False] * self.K
        self._wind_tables()
        for k in range(self.K):
            self._open_episode(k)
            self._write_row(os.path.join(self.dirs[k], "info.csv"), INFO_KEYS, header_only=True)

    # ------------------------------------------------------------------ files
    def _data_file(self, k):
        return os.path.join(self.dirs[k], f"episode_{self.episode[k]}_data.csv")

    @staticmethod
    def _write_row(path, row, header_only=False):
        if header_only and os.path.exists(path):
            return
        with open(path, "x" if header_only else "a", newline="") as f:
            csv.writer(f, delimiter=";").writerow(row)

    def _open_episode(self, k):
        self._write_row(self._data_file(k), COLUMNS, header_only=True)

    def _wind_tables(self):
        """wind.csv: the wind tables of each env's first recorded episode (recorder.py:43-56)."""
        L = int(self.env.cfg.wind_len)
        idx = torch.arange(L, dtype=torch.int32, device=self.env.device)
        self._wind = []
        for i in self.ids_host:
            v, a = self.env.wind_eval(torch.full((L,), i, dtype=torch.int32, device=self.env.device), idx)
            self._wind.append(torch.stack([v, a], 1))

    # ------------------------------------------------------------------ step hooks
    def record(self) -> None:
        """main.py:79 write_data_to_csv: return_all_data() of the state before the step."""
        e, ids = self.env, self.ids
        row = torch.stack([e.s_x[ids], e.s_y[ids], e.v_x[ids], e.v_y[ids], e.s_r[ids],
                           self._last_action, self._last_reward, e.rudder[ids],
                           torch.full_like(self._last_action, N_RPM)], 1)
        self._rows.append(row)

    def after_step(self, actions) -> None:
        """After env.step: the step's action / reward (kept for the next row, like
        BoatEnv.action / .reward) and the episode ends of the sampled envs."""
        e, ids = self.env, self.ids
        a = torch.as_tensor(actions, device=e.device).reshape(-1)
        self._last_action = a[ids].to(torch.float32).to(torch.float64)
        r = e.reward64 if (e.params.out_flags & _lib.OUT_REWARD64) else e.reward
        self._last_reward = r[ids].to(torch.float64)
        c = e.counters[:, ids].to(torch.float64).T                    # [K, 5]
        ev = torch.cat([e.term[ids].to(torch.float64)[:, None],
                        e.final_ep_reward[ids][:, None], c], 1)      # [K, 7]
        self._events.append(ev)
        if len(self._events) >= self.flush_steps:
            self.flush()

    # ------------------------------------------------------------------ host side
    def flush(self) -> None:
        if not self._rows:
            return
        rows = torch.stack(self._rows).cpu().numpy()        # [S, K, 9]
        evs = torch.stack(self._events).cpu().numpy() if self._events else np.zeros((0, self.K, 7))
        self._rows, self._events = [], []
        for s in range(rows.shape[0]):
            for k in range(self.K):
                r = rows[s, k]
                vals = [_fmt(v) for v in r[:5]] + [str(np.float32(r[5])), _fmt(r[6]), _fmt(r[7]),
                                                   str(int(r[8]))]
                self._write_row(self._data_file(k), vals)
                if s < evs.shape[0] and evs[s, k, 0] != 0:
                    self._end_episode(k, evs[s, k])

    def _end_episode(self, k, ev):
        term = int(ev[0])
        name = _lib.TERM_NAMES[term] if term < len(_lib.TERM_NAMES) else str(term)
        info = [name] + [str(int(c)) for c in ev[2:7]] + [_fmt(ev[1])]
        self._write_row(os.path.join(self.dirs[k], "info.csv"), info)       # main.py:100
        if not self._wind_done[k]:                                           # main.py:101
            path = os.path.join(self.dirs[k], "wind.csv")
            if not os.path.exists(path):
                w = self._wind[k].cpu().numpy()
                with open(path, "x", newline="") as f:
                    wr = csv.writer(f, delimiter=";")
                    wr.writerow(["wind_velocity", "wind_angle"])
                    for v, a in w:
                        wr.writerow([_fmt(v), _fmt(a)])
            self._wind_done[k] = True
        self.episode[k] += 1
        self._open_episode(k)

    def close(self) -> None:
        self.flush()


__all__ = ["VecRecorder", "COLUMNS", "INFO_KEYS"]
