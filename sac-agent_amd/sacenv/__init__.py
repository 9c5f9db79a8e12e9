"""sacenv — MI355X-native vectorised boat environment engine.

Hot path of Nilau1998/SAC-Agent (environment/boat_env.py, wind.py,
reward_functions.py, control_theory/control_blocks.py) as gfx950 HIP kernels
behind the reference's Gym surface. See DESIGN.md / INTEGRATION.md.
"""
from . import _lib
from .config import BoatConfig
from .spaces import Box

__all__ = ["BoatConfig", "Box", "VecBoatEnv", "BoatEnv", "ParachuteEnv", "CarEnv", "VecToyEnv",
           "MixedBatch", "_lib"]


def __getattr__(name):  # lazy: importing torch-dependent classes only when used
    if name == "VecBoatEnv":
        from .vec_env import VecBoatEnv
        return VecBoatEnv
    if name == "BoatEnv":
        from .boat_env import BoatEnv
        return BoatEnv
    if name in ("ParachuteEnv", "CarEnv", "VecToyEnv", "MixedBatch"):
        from . import toys
        return getattr(toys, name)
    raise AttributeError(name)
