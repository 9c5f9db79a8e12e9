"""ctypes binding of the C ABI in include/sacenv.h (libsacenv.so, gfx950).

There is no fallback: if the library is missing or a call fails, this module
raises. The product path never computes an env step on the CPU.
"""
from __future__ import annotations

import ctypes as C
import os

from . import _build

PKG_ROOT = _build.PKG_ROOT
LIB_PATH = os.environ.get("SACENV_LIB", _build.LIB)
LOADED_DIGEST = None  # source digest of the loaded library (the in-tree build)

ABI_VERSION = 20
OBS_DIM = 11
MT_N = 624
MAX_KNOTS = 16
N_COUNTERS = 5
SLOTS = 257
REFILL_PERIOD = 256  # autoreset: step launches allowed between sacenv_boat_refill calls
STATUS_SLOT_UNDERFLOW = 1
STATUS_HANDOFF_TIMEOUT = 2
STATUS_LIST_TIMEOUT = 4
FLAG_ABORT = 0xFFFFFFFF  # hand-off flag of a wave / workgroup that gave up (sacenv.h)
RECORD_BYTES = 50
TRANS_OBS = 11          # s' entries in the pooled row (the whole obs)
TRANS_BYTES = 53        # sacenv_boat_step_pooled's per-env transition row
TRANS_BYTES_EXP2 = 57   # experiment 2 (+ obs3_next)


def trans_bytes(experiment: int) -> int:
    """Bytes per env of the pooled transition row for this experiment."""
    return TRANS_BYTES_EXP2 if int(experiment) == 2 else TRANS_BYTES

TERM_NONE, TERM_REACHED_GOAL, TERM_OUT_OF_BOUNDS, TERM_OUT_OF_FUEL, \
    TERM_RUDDER_BROKEN, TERM_TIMEOUT, TERM_TRUNCATED = range(7)
# info-dict key order of the reference (environment/boat_env.py:24-32)
TERM_NAMES = ("", "reached_goal", "out_of_bounds", "out_of_fuel", "rudder_broken",
              "timeout", "truncated")

OUT_ACCEL, OUT_REWARD64, OUT_KNOTS = 1, 2, 4

_d = C.c_double
_i32 = C.c_int32
_i64 = C.c_int64
_p = C.c_void_p


class BoatParams(C.Structure):
    _fields_ = [
        ("n_envs", _i32), ("experiment", _i32), ("test_mode", _i32), ("wind_len", _i32),
        ("n_knots", _i32), ("fuel0", _i32), ("start_y_half", _i32),
        ("max_episode_steps", _i32), ("autoreset", _i32), ("n_helpers", _i32),
        ("out_flags", _i32), ("use_wind_table", _i32),
        ("dt", _d), ("t_max", _d), ("goal_line", _d), ("oob_limit", _d), ("track_width", _d),
        ("c_r_front", _d), ("c_r_side", _d), ("rho", _d), ("boat_area_front", _d),
        ("boat_area_side", _d), ("boat_l", _d), ("boat_b", _d), ("rudder_area", _d),
        ("m_plus_mx", _d), ("m_plus_my", _d), ("i_plus_iz", _d),
        ("one_minus_wf", _d), ("one_minus_td", _d),
        ("n_rpm", _d), ("n_times_d", _d), ("n_squared", _d), ("d_pow4", _d),
        ("max_velocity", _d), ("wind_dir_rad", _d), ("reward_k", _d), ("reward_center", _d),
        ("knot_step", _d), ("knot_inv", _d),
    ]


LAYOUT_FIELDS = (
    "total_bytes", "n_pad", "s_x", "s_y", "s_r", "v_x", "v_y", "v_r", "rudder", "t",
    "ep_reward", "wind_coef", "wind0_next", "start_y_next", "index", "cons", "fill", "mt_pos", "start_y", "counters",
    "refill_list",
    "wind_knots", "knots_raw", "mt_key", "record", "obs", "reward", "done", "term",
    "final_obs", "final_ep_reward", "accel", "reward64", "refill_mask", "status",
    "spline_g", "wind_table", "last_term", "mt_next")


class BoatLayout(C.Structure):
    _fields_ = [(n, _i64) for n in LAYOUT_FIELDS]


TOY_PARACHUTE, TOY_CAR = 1, 2
TOY_TERM_GROUND = 1
TOY_TERM_NAMES = ("", "ground", "", "", "", "timeout", "truncated")


class ToyParams(C.Structure):
    _fields_ = [
        ("n_envs", _i32), ("kind", _i32), ("autoreset", _i32), ("max_episode_steps", _i32),
        ("dt", _d), ("t_max", _d), ("integ_dt", _d),
        ("h0", _d), ("h1", _d), ("area_closed", _d), ("area_open", _d), ("mass", _d),
        ("c_w", _d), ("rho", _d), ("g", _d),
        ("car_accel", _d), ("car_v_max", _d), ("car_dangle", _d),
    ]


TOY_LAYOUT_FIELDS = ("total_bytes", "n_pad", "state", "count", "counters", "record", "obs",
                     "reward", "done", "term", "final_obs")


class ToyLayout(C.Structure):
    _fields_ = [(n, _i64) for n in TOY_LAYOUT_FIELDS]


class ReplayParams(C.Structure):
    _fields_ = [("mem_size", _i64), ("obs_dim", _i32), ("act_dim", _i32), ("reward_f32", _i32),
                ("terminal_mask", C.c_uint32)]


class StagedParams(C.Structure):
    _fields_ = [("period", _i64), ("offset", _i64), ("n", _i32), ("n_pad", _i32), ("seg", _i32),
                ("experiment", _i32), ("first_obs", C.c_float * OBS_DIM)]


class StageSide(C.Structure):
    """SacenvStageSide (sacenv.h): one segment's draws, pack and unpack in one launch."""
    _fields_ = [("draw_g", _i64), ("seed", C.c_uint64), ("draw_idx", _p), ("marks_prev", _p), ("marks_cur", _p),
                ("draw_tiles", _p), ("pack_g", _i64), ("stage_cur", _p), ("stage_prev", _p), ("pack_idx", _p),
                ("pack_tiles", _p), ("cap", _i64), ("chunk", _p), ("gathered", _p), ("chunk_bytes", _i64),
                ("words", _p), ("status_word", _p), ("world", _i32), ("reserved", _i32)]


REPLAY_LAYOUT_FIELDS = ("total_bytes", "state", "new_state", "action", "reward", "terminal",
                        "mem_cntr", "mt_key", "mt_pos")


class ReplayLayout(C.Structure):
    _fields_ = [(n, _i64) for n in REPLAY_LAYOUT_FIELDS]


SAC_HIDDEN = 256


class SacParams(C.Structure):
    _fields_ = [("obs_dim", _i32), ("n_actions", _i32), ("hidden", _i32), ("batch", _i32),
                ("max_action", _d), ("gamma", _d), ("tau", _d), ("reward_scale", _d),
                ("lr_actor", _d), ("lr_critic", _d), ("adam_beta1", _d), ("adam_beta2", _d),
                ("adam_eps", _d)]


class SacLayout(C.Structure):
    _fields_ = [("total_floats", _i64), ("net", _i64 * 5), ("adam_m", _i64 * 4), ("adam_v", _i64 * 4),
                ("w2f", _i64 * 5), ("w2tf", _i64 * 4), ("net_floats", _i64 * 3), ("tensor", (_i64 * 8) * 3),
                ("scratch_bytes", _i64)]


EXPORTS = ("sacenv_abi_version", "sacenv_error_string", "sacenv_boat_layout",
           "sacenv_boat_init", "sacenv_boat_reset", "sacenv_boat_reset_explicit",
           "sacenv_boat_step", "sacenv_boat_step_pooled", "sacenv_boat_rollout", "sacenv_boat_segment",
           "sacenv_boat_segment_occupancy", "sacenv_stream_create_exclusive", "sacenv_stream_destroy",
           "sacenv_boat_refill", "sacenv_boat_wind_eval", "sacenv_toy_layout", "sacenv_toy_init",
           "sacenv_toy_reset", "sacenv_toy_step", "sacenv_mixed_step", "sacenv_mixed_step_pooled",
           "sacenv_mixed_segment", "sacenv_replay_layout",
           "sacenv_replay_init", "sacenv_replay_store", "sacenv_replay_store_env", "sacenv_replay_store_env_at", "sacenv_replay_sample", "sacenv_replay_store_shard",
           "sacenv_replay_sample_shard", "sacenv_replay_stage_scratch_bytes", "sacenv_replay_stage_draw",
           "sacenv_replay_stage_mark", "sacenv_replay_sample_staged", "sacenv_replay_gather",
           "sacenv_replay_stage_draw_ctr", "sacenv_replay_stage_chunk", "sacenv_replay_stage_pack",
           "sacenv_replay_stage_unpack", "sacenv_replay_stage_side", "sacenv_copy_standin",
           "sacenv_compact_done", "sacenv_boat_reset_list", "sacenv_sac_layout", "sacenv_sac_sync",
           "sacenv_sac_act", "sacenv_sac_act_handoff", "sacenv_sac_act_occupancy", "sacenv_sac_learn")

_LIB = None


class SacenvError(RuntimeError):
    pass


def load(path: str | None = None):
    """Load libsacenv.so (once). Raises if it is absent: there is no CPU path."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    global LOADED_DIGEST
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise SacenvError(
            f"libsacenv.so not found at {p}: build it with `python __graft_entry__.py build` "
            "(hipcc --offload-arch=gfx950). The env has no CPU fallback.")
    digest = None
    if os.path.abspath(p) == os.path.abspath(_build.LIB):
        # the in-tree library must be the one the sources in this tree compile to
        digest = _build.source_digest()
        stamp = p + ".sha256"
        have = open(stamp).read().strip() if os.path.exists(stamp) else None
        if have != digest:
            raise SacenvError(
                f"{p} was not built from the sources in this tree (stamp {have and have[:16]}, "
                f"sources {digest[:16]}): rebuild with `python __graft_entry__.py build`")
    # torch first: it brings its own HIP runtime, and the library must bind to
    # that same one (loaded before torch, the library's HIP calls found no
    # device on the MI355X box)
    import torch  # noqa: F401
    lib = C.CDLL(p)
    P = C.POINTER(BoatParams)
    TP = C.POINTER(ToyParams)
    RP = C.POINTER(ReplayParams)
    SP = C.POINTER(StagedParams)
    sig = {
        "sacenv_abi_version": (C.c_int, []),
        "sacenv_error_string": (C.c_char_p, [C.c_int]),
        "sacenv_boat_layout": (C.c_int, [P, C.POINTER(BoatLayout)]),
        "sacenv_boat_init": (C.c_int, [P, _p, _p, _p]),
        "sacenv_boat_reset": (C.c_int, [P, _p, _p, _i32, _p]),
        "sacenv_boat_reset_explicit": (C.c_int, [P, _p, _p, _i32, _p, _p, _p]),
        "sacenv_boat_step": (C.c_int, [P, _p, _p, _p]),
        "sacenv_boat_step_pooled": (C.c_int, [P, _p, _p, _p, _p]),
        "sacenv_boat_refill": (C.c_int, [P, _p, _p]),
        "sacenv_boat_rollout": (C.c_int, [P, _p, _p, _i32, _p, _p, _p]),
        "sacenv_boat_segment": (C.c_int, [P, _p, _p, _i64, _i32, _p, _p, C.c_uint32, _p, _i64, _p, _p, _p]),
        "sacenv_boat_segment_occupancy": (C.c_int, [P, _i32] + [C.POINTER(_i32)] * 4),
        "sacenv_stream_create_exclusive": (C.c_int, [C.POINTER(_p)]),
        "sacenv_stream_destroy": (C.c_int, [_p]),
        "sacenv_boat_wind_eval": (C.c_int, [P, _p, _p, _p, _i32, _p, _p, _p]),
        "sacenv_toy_layout": (C.c_int, [TP, C.POINTER(ToyLayout)]),
        "sacenv_toy_init": (C.c_int, [TP, _p, _p]),
        "sacenv_toy_reset": (C.c_int, [TP, _p, _p, _i32, _p]),
        "sacenv_toy_step": (C.c_int, [TP, _p, _p]),
        "sacenv_mixed_step": (C.c_int, [P, _p, _p, TP, C.POINTER(_p), _i32, _p]),
        "sacenv_mixed_step_pooled": (C.c_int, [P, _p, _p, TP, C.POINTER(_p), _i32, _p, _p]),
        "sacenv_mixed_segment": (C.c_int, [P, _p, _p, _i64, _i32, TP, C.POINTER(_p), _i32, _p]),
        "sacenv_compact_done": (C.c_int, [_p, _i32, _p, _p, _p]),
        "sacenv_boat_reset_list": (C.c_int, [P, _p, _p, _p, _p]),
        "sacenv_replay_layout": (C.c_int, [RP, C.POINTER(ReplayLayout)]),
        "sacenv_replay_init": (C.c_int, [RP, _p, C.c_uint32, _p]),
        "sacenv_replay_store": (C.c_int, [RP, _p, _i64, _p, _p, _p, _p, _p, _p, _p]),
        "sacenv_replay_store_env": (C.c_int, [RP, _p, _i64, _p, _p, _p, _p, _p, _p, _p, _p]),
        "sacenv_replay_store_env_at": (C.c_int, [RP, _p, _i64, _i64, _p, _p, _p, _p, _p, _p, _p, _p]),
        "sacenv_replay_sample": (C.c_int, [RP, _p, _i32, _i64, _p, _p, _p, _p, _p, _p, _p]),
        "sacenv_replay_store_shard": (C.c_int, [RP, _p, _i64, _i64, _i64, _p, _p, _p, _p, _p, _p, _p, _p]),
        "sacenv_replay_sample_shard": (C.c_int, [RP, _p, _i32, _i64, _i64, _i64, _i64, _p, _p, _p, _p, _p, _p,
                                                 _p]),
        "sacenv_replay_stage_scratch_bytes": (C.c_int, [RP, _i32, _i32, C.POINTER(_i64)]),
        "sacenv_replay_stage_draw": (C.c_int, [RP, _p, SP, _i64, _i32, _i32, _p, _p, _i64, _p]),
        "sacenv_replay_stage_mark": (C.c_int, [RP, SP, _i64, _p, _p, _i32, _i32, _p, _p]),
        "sacenv_replay_sample_staged": (C.c_int, [RP, SP, _i64, _p, _p, _p, _i32, _i32, _p, _p]),
        "sacenv_replay_gather": (C.c_int, [RP, _p, _i32, _p, _p, _p, _p, _p, _p, _p]),
        "sacenv_replay_stage_draw_ctr": (C.c_int, [RP, SP, _i64, _i32, _i32, C.c_uint64, _p, _p, _p, _p, _p]),
        "sacenv_replay_stage_chunk": (C.c_int, [RP, SP, _i32, _i32, C.POINTER(_i64), C.POINTER(_i64)]),
        "sacenv_replay_stage_pack": (C.c_int, [RP, SP, _i64, _p, _p, _p, _i32, _i32, _i64, _p, _p, _i32, _p]),
        "sacenv_replay_stage_unpack": (C.c_int, [_i32, _i64, _i64, _i32, _i32, _p, _p, _p, _p]),
        "sacenv_replay_stage_side": (C.c_int, [RP, SP, _i32, _i32, C.POINTER(StageSide), _p]),
        "sacenv_copy_standin": (C.c_int, [_p, _p, _i64, _i32, C.c_double, _p]),
        "sacenv_sac_layout": (C.c_int, [C.POINTER(SacParams), C.POINTER(SacLayout)]),
        "sacenv_sac_sync": (C.c_int, [C.POINTER(SacParams), _p, _p]),
        "sacenv_sac_act": (C.c_int, [C.POINTER(SacParams), _p, _p, _i32, _p, _p, _p, _p]),
        "sacenv_sac_act_handoff": (C.c_int, [C.POINTER(SacParams), _p, _p, _i32, _p, _p, _p, C.c_uint32, _p,
                                             C.c_uint32, _p, _p]),
        "sacenv_sac_act_occupancy": (C.c_int, [_i32] + [C.POINTER(_i32)] * 4),
        "sacenv_sac_learn": (C.c_int, [C.POINTER(SacParams), _p, _p, _p, _p, _p, _p, _p, _p, _p, _i32,
                                       _p, _p]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype, f.argtypes = res, args
    v = lib.sacenv_abi_version()
    if v != ABI_VERSION:
        raise SacenvError(f"libsacenv ABI {v} != expected {ABI_VERSION}")
    if path is None:
        _LIB = lib
        LOADED_DIGEST = digest
    return lib


def check(rc: int) -> None:
    if rc != 0:
        msg = load().sacenv_error_string(rc).decode()
        if rc in (-2, -3, -5):
            raise ValueError(msg)
        raise SacenvError(f"sacenv call failed ({rc}): {msg}")


def layout(params: BoatParams) -> BoatLayout:
    out = BoatLayout()
    check(load().sacenv_boat_layout(C.byref(params), C.byref(out)))
    return out


def toy_layout(params: ToyParams) -> ToyLayout:
    out = ToyLayout()
    check(load().sacenv_toy_layout(C.byref(params), C.byref(out)))
    return out


def sac_layout(params: SacParams) -> SacLayout:
    out = SacLayout()
    check(load().sacenv_sac_layout(C.byref(params), C.byref(out)))
    return out


def replay_layout(params: ReplayParams) -> ReplayLayout:
    out = ReplayLayout()
    check(load().sacenv_replay_layout(C.byref(params), C.byref(out)))
    return out
