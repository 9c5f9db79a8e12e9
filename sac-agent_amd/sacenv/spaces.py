"""Gym space used by the env surface.

The reference's agent does ``isinstance(env.action_space, gym.spaces.Box)``
(agent/base_agent.py:9,16), so gym's own ``Box`` is used whenever gym is
importable; otherwise a minimal class with the attributes the reference
reads (``shape``, ``high``, ``low``, ``dtype``) stands in.
"""
from __future__ import annotations

import numpy as np

try:  # pragma: no cover - gym is absent in this image
    from gym.spaces import Box  # type: ignore
except Exception:  # noqa: BLE001
    try:  # pragma: no cover
        from gymnasium.spaces import Box  # type: ignore
    except Exception:  # noqa: BLE001

        class Box:  # type: ignore[no-redef]
            """gym-0.26 ``Box`` semantics: scalar bounds -> shape (1,)."""

            def __init__(self, low, high, shape=None, dtype=np.float32):
                dtype = np.dtype(dtype)
                low_a, high_a = np.asarray(low, dtype), np.asarray(high, dtype)
                if shape is None:
                    shape = low_a.shape if low_a.shape != () else (1,)
                self.shape = tuple(int(s) for s in shape)
                self.dtype = dtype
                self.low = np.broadcast_to(low_a, self.shape).astype(dtype)
                self.high = np.broadcast_to(high_a, self.shape).astype(dtype)

            def sample(self):
                return np.random.uniform(self.low, self.high).astype(self.dtype)

            def contains(self, x) -> bool:
                x = np.asarray(x)
                return x.shape == self.shape and bool(np.all(x >= self.low) & np.all(x <= self.high))

            def __repr__(self) -> str:
                return f"Box({self.low}, {self.high}, {self.shape}, {self.dtype})"
