"""Import the read-only reference (Nilau1998/SAC-Agent) in THIS container only.

Test infrastructure, not product code: used solely by ``make_golden.py`` to
produce the committed ``.npz`` fixtures. The reference never travels to the
GPU box and nothing under ``sac-agent_amd/`` imports this file.

The reference needs ``gym``, ``dotmap`` and ``seaborn``, none of which is
installed here. They are replaced by minimal ``sys.modules`` stand-ins with
the semantics the reference relies on:

* ``gym.Env``          - empty base class (``boat_env.py:9``)
* ``gym.spaces.Box``   - gym-0.26 shape rule: scalar low/high -> shape (1,)
                          (``boat_env.py:37-41``)
* ``dotmap.DotMap``    - recursive attribute dict (``utils/config_reader.py:6-8``)
* ``seaborn``          - no-op plotting functions (``control_blocks.py:2``,
                          ``reward_functions.py:5``)
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np
import yaml

REF_ROOT = os.environ.get("SACENV_REFERENCE", "/root/reference")


class _DotMap(dict):
    def __init__(self, d=None):
        super().__init__()
        for k, v in (d or {}).items():
            self[k] = _DotMap(v) if isinstance(v, dict) else v

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:  # pragma: no cover
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v


class _Box:
    def __init__(self, low, high, shape=None, dtype=np.float32):
        low = np.asarray(low, dtype=dtype)
        high = np.asarray(high, dtype=dtype)
        if shape is None:
            shape = low.shape if low.shape != () else (1,)
        self.shape = tuple(shape)
        self.low = np.broadcast_to(low, self.shape).astype(dtype)
        self.high = np.broadcast_to(high, self.shape).astype(dtype)
        self.dtype = np.dtype(dtype)


def install_standins() -> None:
    if "gym" not in sys.modules:
        gym = types.ModuleType("gym")
        gym.Env = type("Env", (), {})
        spaces = types.ModuleType("gym.spaces")
        spaces.Box = _Box
        gym.spaces = spaces
        sys.modules["gym"] = gym
        sys.modules["gym.spaces"] = spaces
    if "dotmap" not in sys.modules:
        dm = types.ModuleType("dotmap")
        dm.DotMap = _DotMap
        sys.modules["dotmap"] = dm
    if "seaborn" not in sys.modules:
        sns = types.ModuleType("seaborn")
        for name in ("set_style", "lineplot", "despine", "set_theme"):
            setattr(sns, name, lambda *a, **k: None)
        sys.modules["seaborn"] = sns
    sys.dont_write_bytecode = True
    if REF_ROOT not in sys.path:
        sys.path.insert(0, REF_ROOT)


def load_config(overrides: dict | None = None) -> _DotMap:
    """``configs/original_config.yaml`` + nested overrides, as a DotMap."""
    with open(os.path.join(REF_ROOT, "configs", "original_config.yaml")) as f:
        raw = yaml.safe_load(f)
    for sect, kv in (overrides or {}).items():
        raw.setdefault(sect, {}).update(kv)
    return _DotMap(raw)


def boat_env_module():
    install_standins()
    import environment.boat_env as be  # noqa: E402  (reference module)
    return be
