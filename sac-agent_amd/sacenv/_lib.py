"""ctypes binding of the C ABI in include/sacenv.h (libsacenv.so, gfx950).

There is no fallback: if the library is missing or a call fails, this module
raises. The product path never computes an env step on the CPU.
"""
from __future__ import annotations

import ctypes as C
import os

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # .../sac-agent_amd
LIB_PATH = os.environ.get("SACENV_LIB", os.path.join(PKG_ROOT, "build", "libsacenv.so"))

ABI_VERSION = 1
OBS_DIM = 11
MT_N = 624
MAX_KNOTS = 16
N_COUNTERS = 5

TERM_NONE, TERM_REACHED_GOAL, TERM_OUT_OF_BOUNDS, TERM_OUT_OF_FUEL, \
    TERM_RUDDER_BROKEN, TERM_TIMEOUT, TERM_TRUNCATED = range(7)
# info-dict key order of the reference (environment/boat_env.py:24-32)
TERM_NAMES = ("", "reached_goal", "out_of_bounds", "out_of_fuel", "rudder_broken",
              "timeout", "truncated")

_d = C.c_double
_i32 = C.c_int32
_pd = C.c_void_p


class BoatParams(C.Structure):
    _fields_ = [
        ("n_envs", _i32), ("experiment", _i32), ("test_mode", _i32), ("wind_len", _i32),
        ("n_knots", _i32), ("fuel0", _i32), ("start_y_half", _i32),
        ("max_episode_steps", _i32), ("autoreset", _i32), ("reserved0", _i32),
        ("dt", _d), ("t_max", _d), ("goal_line", _d), ("oob_limit", _d), ("track_width", _d),
        ("boat_m", _d), ("boat_m_x", _d), ("boat_m_y", _d), ("boat_I", _d), ("boat_Iz", _d),
        ("propeller_diameter", _d), ("wake_friction", _d), ("c_r_front", _d), ("c_r_side", _d),
        ("thrust_deduction", _d), ("rho", _d),
        ("boat_area_front", _d), ("boat_area_side", _d), ("boat_l", _d), ("boat_b", _d),
        ("rudder_area", _d),
        ("n_rpm", _d), ("max_velocity", _d), ("wind_dir_rad", _d), ("reward_k", _d),
        ("reward_center", _d), ("knot_step", _d),
        ("obs_lo", _d * OBS_DIM), ("obs_hi", _d * OBS_DIM),
        ("spline_g", _pd), ("wind_table", _pd),
    ]


class BoatState(C.Structure):
    _fields_ = [(n, _pd) for n in (
        "s_x", "s_y", "s_r", "v_x", "v_y", "v_r", "rudder", "t", "ep_reward",
        "index", "start_y", "wind_y", "wind_m", "knots_raw", "mt_key", "mt_pos", "counters")]


class BoatStepOut(C.Structure):
    _fields_ = [(n, _pd) for n in (
        "obs", "reward", "done", "term", "final_obs", "final_ep_reward", "accel", "reward64")]


EXPORTS = ("sacenv_abi_version", "sacenv_error_string", "sacenv_boat_seed",
           "sacenv_boat_reset", "sacenv_boat_reset_explicit", "sacenv_boat_step",
           "sacenv_boat_wind_eval")

_LIB = None


class SacenvError(RuntimeError):
    pass


def load(path: str | None = None):
    """Load libsacenv.so (once). Raises if it is absent: there is no CPU path."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise SacenvError(
            f"libsacenv.so not found at {p}: build it with `python __graft_entry__.py build` "
            "(hipcc --offload-arch=gfx950). The env has no CPU fallback.")
    lib = C.CDLL(p)
    P, S, O = C.POINTER(BoatParams), C.POINTER(BoatState), C.POINTER(BoatStepOut)
    lib.sacenv_abi_version.restype = C.c_int
    lib.sacenv_abi_version.argtypes = []
    lib.sacenv_error_string.restype = C.c_char_p
    lib.sacenv_error_string.argtypes = [C.c_int]
    lib.sacenv_boat_seed.restype = C.c_int
    lib.sacenv_boat_seed.argtypes = [P, S, _pd, _pd]
    lib.sacenv_boat_reset.restype = C.c_int
    lib.sacenv_boat_reset.argtypes = [P, S, _pd, _i32, _pd, _pd]
    lib.sacenv_boat_reset_explicit.restype = C.c_int
    lib.sacenv_boat_reset_explicit.argtypes = [P, S, _pd, _i32, _pd, _pd, _pd, _pd]
    lib.sacenv_boat_step.restype = C.c_int
    lib.sacenv_boat_step.argtypes = [P, S, _pd, O, _pd]
    lib.sacenv_boat_wind_eval.restype = C.c_int
    lib.sacenv_boat_wind_eval.argtypes = [P, S, _pd, _pd, _i32, _pd, _pd, _pd]
    v = lib.sacenv_abi_version()
    if v != ABI_VERSION:
        raise SacenvError(f"libsacenv ABI {v} != expected {ABI_VERSION}")
    if path is None:
        _LIB = lib
    return lib


def check(rc: int) -> None:
    if rc != 0:
        msg = load().sacenv_error_string(rc).decode()
        if rc == -2:
            raise ValueError(msg)
        if rc in (-3, -5):
            raise ValueError(msg)
        raise SacenvError(f"sacenv call failed ({rc}): {msg}")
