"""CPU-only checks of the host side and of the algorithms the kernels implement.

* the C-ABI library loads and exports every entry point include/sacenv.h
  declares; the ctypes mirrors have the C layout (gcc offsetof probe);
* the numpy-legacy MT19937 algorithm the reset kernel implements — seeding,
  the four-phase lane-parallel twist, tempering, masked-rejection randint,
  53-bit doubles — reproduces ``np.random.RandomState`` word for word;
* the not-a-knot spline in second-derivative form (config.spline_g) equals
  scipy's interp1d basis the reference uses (wind.py:82-84), and the
  critical-point grid min/max rule the reset kernel uses finds the exact
  grid extrema.
No compute call is made into the library here (no GPU in this container).
"""
import ctypes
import math
import os
import re
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "sacenv.h")


def declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"\b(sacenv_\w+)\s*\(", src)))


def test_library_exports_header(built_lib):
    from sacenv import _lib
    names = declared_functions()
    assert len(names) == 49
    assert set(names) == set(_lib.EXPORTS)
    for n in names:
        assert hasattr(built_lib, n), n
    assert built_lib.sacenv_abi_version() == _lib.ABI_VERSION
    assert built_lib.sacenv_error_string(-2).decode().startswith("Well someone")


def test_staged_sampler_argument_errors_without_gpu(built_lib):
    """sacenv_replay_stage_draw / _stage_mark / _sample_staged validate on the host, never launching."""
    from sacenv import _lib
    rp = _lib.ReplayParams(mem_size=1_000_000, obs_dim=11, act_dim=1, reward_f32=1, terminal_mask=2)
    sp = _lib.StagedParams(period=4096, offset=0, n=4096, n_pad=4096, seg=256, experiment=6)
    R, S = ctypes.byref(rp), ctypes.byref(sp)
    gather = (0, 1, 1, 1, 1024, 256, 1, None)
    sp.period = sp.n = sp.n_pad = 64      # mem_size > seg * period: a learn could reach older rows
    assert built_lib.sacenv_replay_sample_staged(R, S, *gather) == -5
    assert built_lib.sacenv_replay_stage_draw(R, 1, S, 0, 1024, 256, 1, 1, 1 << 30, None) == -5
    sp.period = sp.n = sp.n_pad = 4096
    rp.obs_dim = 10                       # the boat's rows only
    assert built_lib.sacenv_replay_sample_staged(R, S, *gather) == -4
    rp.obs_dim = 11
    sp.n_pad = 4000                       # not a multiple of 64
    assert built_lib.sacenv_replay_stage_mark(R, S, 0, 1, 1, 1024, 256, 1, None) == -4
    sp.n_pad, sp.offset = 4096, 1         # offset + n > period
    assert built_lib.sacenv_replay_stage_mark(R, S, 0, 1, 1, 1024, 256, 1, None) == -5
    sp.offset = 0
    assert built_lib.sacenv_replay_stage_mark(R, S, 0, None, 1, 1024, 256, 1, None) == -1
    assert built_lib.sacenv_replay_sample_staged(R, S, 0, None, 1, 1, 1024, 256, 1, None) == -1
    assert built_lib.sacenv_replay_stage_draw(R, None, S, 0, 1024, 256, 1, 1, 1 << 30, None) == -1
    # steady state (g >= 1 here) needs the scratch the library asks for
    need = ctypes.c_int64()
    assert built_lib.sacenv_replay_stage_scratch_bytes(R, 1024, 256, ctypes.byref(need)) == 0
    assert need.value > 4 * 624 * 256 * 1024 / 0.95 / 624
    assert built_lib.sacenv_replay_stage_draw(R, 1, S, 300, 1024, 256, 1, 1, need.value - 1, None) == -4


def test_counter_sampler_and_allgather_argument_errors_without_gpu(built_lib):
    """The round-6 entry points (counter-based draws, the all-gather's pack / unpack, the
    collective stand-in, the gather at given indices) validate on the host, never launching."""
    from sacenv import _lib
    rp = _lib.ReplayParams(mem_size=1_000_000, obs_dim=11, act_dim=1, reward_f32=1, terminal_mask=2)
    sp = _lib.StagedParams(period=4096, offset=0, n=4096, n_pad=4096, seg=256, experiment=6)
    R, S = ctypes.byref(rp), ctypes.byref(sp)
    assert built_lib.sacenv_replay_stage_draw_ctr(R, S, 0, 1024, 256, 0, None, None, None, None, None) == -1
    assert built_lib.sacenv_replay_stage_draw_ctr(R, S, 0, 1024, 257, 0, 1, None, None, None, None) == -4
    assert built_lib.sacenv_replay_stage_draw_ctr(R, S, -1, 1024, 256, 0, 1, None, None, None, None) == -4
    sp.period = sp.n = sp.n_pad = 64      # mem_size > seg * period
    assert built_lib.sacenv_replay_stage_draw_ctr(R, S, 0, 1024, 256, 0, 1, None, None, None, None) == -5
    sp.period = sp.n = sp.n_pad = 4096
    assert built_lib.sacenv_replay_stage_pack(R, S, 0, 16, 16, 8, 1024, 256, 10, None, 4, 0, None) == -1
    assert built_lib.sacenv_replay_stage_pack(R, S, 0, 16, 16, 8, 1024, 256, 10, 16, None, 0, None) == -1
    assert built_lib.sacenv_replay_stage_pack(R, S, 0, 24, 16, 8, 1024, 256, 10, 16, 4, 0, None) == -5
    cap, nb = ctypes.c_int64(), ctypes.c_int64()
    assert built_lib.sacenv_replay_stage_chunk(R, S, 1024, 256, ctypes.byref(cap), ctypes.byref(nb)) == 0
    assert cap.value == 1024 * 256 and nb.value >= 16 + 100 * cap.value
    sp.period = 3 * 4096 - 1              # not world x n
    assert built_lib.sacenv_replay_stage_chunk(R, S, 1024, 256, ctypes.byref(cap), ctypes.byref(nb)) == -5
    assert built_lib.sacenv_replay_stage_unpack(2, 16 + 100 * 10 - 4, 10, 64, 4, 16, 16, 16, None) == -4
    assert built_lib.sacenv_replay_stage_unpack(2, 16 + 100 * 10, 10, 64, 4, None, 16, 16, None) == -1
    assert built_lib.sacenv_replay_stage_unpack(0, 16 + 100 * 10, 10, 64, 4, 16, 16, 16, None) == -4
    assert built_lib.sacenv_copy_standin(16, 32, 17, 16, 0.0, None) == -4        # 16-B multiple
    assert built_lib.sacenv_copy_standin(16, 32, 32, 0, 0.0, None) == -4         # workgroups
    assert built_lib.sacenv_copy_standin(16, 32, 32, 16, 2e5, None) == -4        # resident time bound
    assert built_lib.sacenv_copy_standin(None, 32, 32, 16, 1.0, None) == -1
    assert built_lib.sacenv_copy_standin(8, 32, 32, 16, 1.0, None) == -5         # alignment
    assert built_lib.sacenv_replay_gather(R, 1, 4, None, None, None, None, None, None, None) == -1


def test_stage_side_argument_errors_without_gpu(built_lib):
    """sacenv_replay_stage_side (ABI 20: one segment's draws, pack and unpack in one launch)
    validates each role's arguments and refuses buffers the side-by-side roles would share."""
    from sacenv import _lib
    rp = _lib.ReplayParams(mem_size=1_000_000, obs_dim=11, act_dim=1, reward_f32=1, terminal_mask=2)
    sp = _lib.StagedParams(period=4096, offset=0, n=4096, n_pad=4096, seg=256, experiment=6)
    R, S = ctypes.byref(rp), ctypes.byref(sp)
    side = built_lib.sacenv_replay_stage_side
    assert side(R, S, 1024, 256, None, None) == -1
    w = _lib.StageSide(draw_g=2, pack_g=-1, gathered=None)
    assert side(R, S, 1024, 256, ctypes.byref(w), None) == -1           # draws without idx
    w.draw_idx, w.marks_cur, w.draw_tiles = 256, 512, 768
    w.draw_g = -3
    w.pack_g = 0
    assert side(R, S, 1024, 256, ctypes.byref(w), None) == -1           # pack without its buffers
    w.stage_cur, w.stage_prev, w.pack_idx, w.pack_tiles, w.chunk = 1024, 2048, 4096, 8192, 1 << 20
    w.cap = 1024 * 256 + 1                                              # more records than slots
    assert side(R, S, 1024, 256, ctypes.byref(w), None) == -4
    w.cap = 1024 * 256
    w.draw_g, w.draw_idx = 2, 4096                                      # the pack reads what the draws write
    assert side(R, S, 1024, 256, ctypes.byref(w), None) == -5
    w.draw_idx = 256
    w.stage_cur = 1032                                                  # rows not 16-B aligned
    assert side(R, S, 1024, 256, ctypes.byref(w), None) == -5
    w.stage_cur = 1024
    w.gathered, w.world, w.words, w.status_word = (1 << 20) + 64, 1, 1 << 30, 64
    w.chunk_bytes = 16 + 100 * w.cap - 4                                # chunk too small for cap
    assert side(R, S, 1024, 256, ctypes.byref(w), None) == -4
    w.chunk_bytes = 16 + 100 * w.cap
    assert side(R, S, 1024, 256, ctypes.byref(w), None) == -5           # unpacks the chunk being packed
    w.world = 0
    assert side(R, S, 1024, 256, ctypes.byref(w), None) == -4
    w.world, w.draw_g = 1, -1
    sp.period = sp.n = sp.n_pad = 64                                    # mem_size > seg * period
    assert side(R, S, 1024, 256, ctypes.byref(w), None) == -5


def test_segment_marks_are_bounded_without_autoreset(built_lib):
    """the segment launch stages one mark word per step in LDS (256 of them): with
    stage marks, n_steps > SACENV_REFILL_PERIOD is refused in any autoreset mode."""
    from sacenv.config import BoatConfig, make_params
    p = make_params(BoatConfig(experiment=6), 64)
    p.autoreset = 0
    seg = built_lib.sacenv_boat_segment
    assert seg(ctypes.byref(p), 1, 1, 64, 257, None, None, 0, None, 0, 4096, 8, None) == -4
    assert seg(ctypes.byref(p), None, 1, 64, 256, None, None, 0, None, 0, 4096, 8, None) == -1


def test_argument_errors_without_gpu(built_lib):
    """Argument validation runs on the host and never launches."""
    from sacenv.config import BoatConfig, make_params
    p = make_params(BoatConfig(experiment=6), 4)
    p.experiment = 7
    assert built_lib.sacenv_boat_step(ctypes.byref(p), None, None, None) == -2
    p.experiment = 6
    assert built_lib.sacenv_boat_step(ctypes.byref(p), None, None, None) == -1
    p.n_knots = 3
    assert built_lib.sacenv_boat_step(ctypes.byref(p), None, None, None) == -3
    p.n_knots = 8
    p.start_y_half = 0
    assert built_lib.sacenv_boat_step(ctypes.byref(p), None, None, None) == -5
    p.start_y_half = 640
    p.autoreset = 1
    p.n_helpers = 0
    assert built_lib.sacenv_boat_step(ctypes.byref(p), None, None, None) == -4
    p.n_helpers = 256
    p.autoreset = 1
    assert built_lib.sacenv_boat_reset_explicit(ctypes.byref(p), 1, 1, 1, 1, None, None) == -6
    assert built_lib.sacenv_boat_refill(ctypes.byref(p), None, None) == -1
    p.autoreset = 0
    assert built_lib.sacenv_boat_refill(ctypes.byref(p), 1, None) == -6
    # 32-bit byte offsets into wind_knots: n_pad x SLOTS x 2 x knots x 16 B < 2**32
    p.n_knots = 16
    p.n_envs = (1 << 22) + 1  # 32-bit per-env field offsets (no slot-ring cap since round 2)
    assert built_lib.sacenv_boat_step(ctypes.byref(p), 1, 1, None) == -4
    p.n_envs = 1 << 15
    assert built_lib.sacenv_boat_step(ctypes.byref(p), None, None, None) == -1


def test_toy_argument_errors_without_gpu(built_lib):
    from sacenv import _lib
    from sacenv.toys import ParachuteConfig, make_toy_params
    p = make_toy_params(_lib.TOY_PARACHUTE, ParachuteConfig(), 4)
    assert built_lib.sacenv_toy_step(ctypes.byref(p), None, None) == -1
    p.kind = 3
    assert built_lib.sacenv_toy_step(ctypes.byref(p), None, None) == -2
    p.kind = _lib.TOY_CAR
    p.n_envs = 0
    assert built_lib.sacenv_toy_init(ctypes.byref(p), None, None) == -4
    p.n_envs = 4
    assert built_lib.sacenv_mixed_step(None, None, None, ctypes.byref(p), None, 3, None) == -4
    assert built_lib.sacenv_mixed_step(None, None, None, None, None, 1, None) == -1


@pytest.mark.parametrize("n", [1, 63, 64, 32768])
def test_toy_layout(built_lib, n):
    from sacenv import _lib
    from sacenv.toys import CarConfig, make_toy_params
    L = _lib.toy_layout(make_toy_params(_lib.TOY_CAR, CarConfig(), n))
    np_ = L.n_pad
    assert np_ % 64 == 0 and n <= np_ < n + 64
    sizes = {"state": 40, "count": 4, "counters": 12, "obs": 8, "reward": 4, "done": 1, "term": 1,
             "final_obs": 8}
    spans = sorted((getattr(L, f), getattr(L, f) + w * np_, f) for f, w in sizes.items())
    for (a0, a1, f), (b0, b1, g) in zip(spans, spans[1:]):
        assert a1 <= b0, (f, g)
    assert L.record == L.obs and L.term + np_ == L.record + 14 * np_
    assert spans[-1][1] <= L.total_bytes


def test_ctypes_structs_match_c_layout(tmp_path):
    """offsetof/sizeof of every ABI struct, from gcc on include/sacenv.h, vs the ctypes mirrors."""
    from sacenv import _lib
    structs = {"SacenvBoatParams": _lib.BoatParams, "SacenvBoatLayout": _lib.BoatLayout,
               "SacenvToyParams": _lib.ToyParams, "SacenvToyLayout": _lib.ToyLayout,
               "SacenvReplayParams": _lib.ReplayParams, "SacenvReplayLayout": _lib.ReplayLayout,
               "SacenvSacParams": _lib.SacParams, "SacenvSacLayout": _lib.SacLayout,
               "SacenvStagedParams": _lib.StagedParams, "SacenvStageSide": _lib.StageSide}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "sacenv.h"', "int main(void) {"]
    for cname, py in structs.items():
        lines.append(f'printf("{cname} sizeof %zu\\n", sizeof({cname}));')
        for fname, _ in py._fields_:
            lines.append(f'printf("{cname} {fname} %zu\\n", offsetof({cname}, {fname}));')
    lines.append("return 0; }")
    src = tmp_path / "probe.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)],
                   check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    got = {tuple(l.split()[:2]): int(l.split()[2]) for l in out if l.strip()}
    for cname, py in structs.items():
        assert got[(cname, "sizeof")] == ctypes.sizeof(py), cname
        for fname, _ in py._fields_:
            assert got[(cname, fname)] == getattr(py, fname).offset, (cname, fname)


@pytest.mark.parametrize("n,knots", [(1, False), (63, True), (64, False), (65536, False), (65536, True),
                                     (100000, False)])
def test_arena_layout(built_lib, n, knots):
    """Fields are aligned, disjoint and inside total_bytes; record is contiguous; the
    drawn knots get storage only when recorded (SACENV_OUT_KNOTS)."""
    from sacenv import _lib
    from sacenv.config import BoatConfig, make_params
    p = make_params(BoatConfig(experiment=6), n, use_wind_table=True,
                    out_flags=_lib.OUT_KNOTS if knots else 0)
    L = _lib.layout(p)
    np_ = L.n_pad
    assert np_ % 64 == 0 and n <= np_ < n + 64
    nk = 8
    S = _lib.SLOTS
    # paired f64 fields: [n_pad][2] blocks, the second element 8 B after the first
    for a, b in (("s_x", "s_y"), ("s_r", "v_x"), ("v_y", "v_r"), ("rudder", "ep_reward")):
        assert getattr(L, b) == getattr(L, a) + 8, (a, b)
    sizes = {"s_x": 16, "s_r": 16, "v_y": 16, "rudder": 16, "t": 8,
             "wind_coef": 64, "wind0_next": 16, "start_y_next": 4,
             "index": 4, "cons": 4, "fill": 4, "mt_pos": 4,
             "start_y": 4 * S, "counters": 20, "refill_list": 12, "wind_knots": 32 * S * nk,
             "mt_key": 2496, "mt_next": 2496, "obs": 44, "reward": 4, "done": 1, "term": 1,
             "final_obs": 44, "final_ep_reward": 8, "accel": 24, "reward64": 8, "last_term": 4}
    if knots:
        sizes["knots_raw"] = 16 * S * nk
    else:
        assert L.knots_raw == -1
    spans = sorted((getattr(L, f), getattr(L, f) + w * np_, f) for f, w in sizes.items())
    for (a0, a1, f), (b0, b1, g) in zip(spans, spans[1:]):
        assert a1 <= b0, (f, g)
    for a0, a1, f in spans:
        assert a0 % 64 == 0, f
    assert L.record == L.obs and L.term + np_ == L.record + 50 * np_
    tail = [("refill_mask", 8 * np_ // 64), ("status", 256),
            ("spline_g", 8 * 256), ("wind_table", 16 * 10000)]
    end = spans[-1][1]
    for f, w in tail:
        off = getattr(L, f)
        assert off >= end and off % 256 == 0, f
        end = off + w
    assert end <= L.total_bytes
    if n == 65536:   # per env: the wind slots dominate (<= 75 KB without recorded knots)
        per_env = (L.total_bytes - 16 * 10000) / n
        assert per_env <= (106 * 1024 if knots else 73 * 1024), per_env


# ---------------------------------------------------------------- MT19937
M32 = 0xFFFFFFFF


def mt_seed(seed):
    key = [0] * 624
    x = seed & M32
    for i in range(624):
        key[i] = x
        x = (1812433253 * (x ^ (x >> 30)) + i + 1) & M32
    return key, 624


def mix(a, b, c):
    y = (a & 0x80000000) | (b & 0x7FFFFFFF)
    return c ^ (y >> 1) ^ (0x9908B0DF if y & 1 else 0)


def twist_phased(o):
    """Exactly the kernel's mt_twist_wave phase split (lane-parallel phases)."""
    n = [None] * 624
    for i in range(0, 227):
        n[i] = mix(o[i], o[i + 1], o[i + 397])
    for i in range(227, 454):
        n[i] = mix(o[i], o[i + 1], n[i - 227])
    for i in range(454, 623):
        n[i] = mix(o[i], o[i + 1], n[i - 227])
    n[623] = mix(o[623], n[0], n[396])
    return n


def temper(y):
    y ^= y >> 11
    y ^= (y << 7) & 0x9D2C5680
    y ^= (y << 15) & 0xEFC60000
    y ^= y >> 18
    return y & M32


class PyMT:
    def __init__(self, seed):
        self.key, self.pos = mt_seed(seed)

    def next32(self):
        if self.pos >= 624:
            self.key, self.pos = twist_phased(self.key), 0
        w = self.key[self.pos]
        self.pos += 1
        return temper(w)

    def randint(self, lo, hi):
        rng = hi - 1 - lo
        mask = rng
        for s in (1, 2, 4, 8, 16):
            mask |= mask >> s
        while True:
            v = self.next32() & mask
            if v <= rng:
                return lo + v

    def sample(self):
        a, b = self.next32() >> 5, self.next32() >> 6
        return (a * 67108864.0 + b) / 9007199254740992.0


@pytest.mark.parametrize("seed", [0, 1, 12345, 2**31 + 11, 2**32 - 1])
def test_mt19937_matches_numpy_legacy(seed):
    ref = np.random.RandomState(seed)
    me = PyMT(seed)
    for _ in range(40):  # 40 Boat resets of exp 6: crosses several 624-word blocks
        assert me.randint(-640, 640) == ref.randint(-640, 640)
        kv = [me.sample() for _ in range(16)]
        assert kv == list(ref.random_sample(16))
    st = ref.get_state()
    assert list(st[1]) == me.key and st[2] == me.pos


# ---------------------------------------------------------------- spline
def test_spline_g_equals_scipy_basis():
    from boat_oracle import spline_basis
    from sacenv.config import spline_g
    for L, n in ((10000, 8), (20, 8), (500, 4), (10000, 16)):
        B = spline_basis(L, n)
        G = spline_g(n)
        r = (n - 1) / (L - 1)
        i = np.arange(L)
        s = i * r
        j = np.minimum(s.astype(int), n - 2)
        t = s - j
        u = 1 - t
        E = np.eye(n)
        # basis functions through the second-derivative form
        M = G @ E
        val = (u[:, None] * E[j] + t[:, None] * E[j + 1]
               + (u ** 3 - u)[:, None] * M[j] + (t ** 3 - t)[:, None] * M[j + 1])
        np.testing.assert_allclose(val, B, rtol=0, atol=2e-14)


def _interval_extrema_py(y, m, n, L, j):
    """Python mirror of the kernel's interval_extrema candidate rule -> grid indices."""
    step = (n - 1) / (L - 1)
    jf = lambda i: min(int(i * step), n - 2)

    inv = (L - 1) / (n - 1)        # the host's knot_inv (sacenv/config.py)
    lo = max(math.ceil(j * inv) - 1, 0)
    while lo < L and jf(lo) < j:
        lo += 1
    hi = min(math.floor((j + 1) * inv) + 1, L - 1)
    while hi >= 0 and jf(hi) > j:
        hi -= 1
    if lo > hi:
        return [], []
    cand = [lo, hi]
    a, b = m[j], m[j + 1]
    qa, qb, qc = 3 * (b - a), 6 * a, y[j + 1] - y[j] - 2 * a - b
    roots = []
    scale = abs(qa) + abs(qb) + abs(qc)
    if abs(qa) <= 1e-14 * scale:
        if qb != 0:
            roots.append(-qc / qb)
    else:
        disc = qb * qb - 4 * qa * qc
        if disc >= 0:
            q = -0.5 * (qb + math.copysign(math.sqrt(disc), qb if qb != 0 else 1.0))
            roots.append(q / qa)
            if q != 0:
                roots.append(qc / q)
    for tr in roots:
        if not (-0.01 < tr < 1.01):
            continue
        i0 = math.floor((j + tr) * inv)
        for d in (-1, 0, 1, 2):
            cand.append(min(max(i0 + d, lo), hi))
    return cand, (lo, hi)


def test_interval_bound_starts_never_overshoot():
    """interval_extrema starts its first/last grid-index searches one below ceil(j inv)
    and one above floor((j+1) inv) and only walks inward from there: exhaustively, for
    4..16 knots and every L up to 20 000, neither start lies past the true bound."""
    bad = 0
    for n in range(4, 17):
        for L in range(n, 20001):
            step, inv = (n - 1) / (L - 1), (L - 1) / (n - 1)
            jf = lambda i: min(int(i * step), n - 2)  # noqa: E731
            for j in range(n - 1):
                lo0 = max(math.ceil(j * inv) - 1, 0)
                i = max(lo0 - 5, 0)
                while jf(i) < j:
                    i += 1
                hi0 = min(math.floor((j + 1) * inv) + 1, L - 1)
                k = min(hi0 + 5, L - 1)
                while k >= 0 and jf(k) > j:
                    k -= 1
                bad += lo0 > i or hi0 < k
    assert bad == 0


@pytest.mark.parametrize("L", [10000, 20, 37])
def test_grid_extrema_rule_is_exact(L):
    from sacenv.config import spline_g
    rng = np.random.RandomState(3)
    n = 8
    G = spline_g(n)
    step = (n - 1) / (L - 1)
    for _ in range(300):
        y = rng.random_sample(n)
        m = G @ y
        i = np.arange(L)
        s = i * step
        jj = np.minimum(s.astype(int), n - 2)
        t = s - jj
        u = 1 - t
        full = u * y[jj] + t * y[jj + 1] + (u * u * u - u) * m[jj] + (t * t * t - t) * m[jj + 1]
        cands, cover = [], 0
        for j in range(n - 1):
            cand, rng_ = _interval_extrema_py(y, m, n, L, j)
            cands += cand
            if rng_:
                cover += rng_[1] - rng_[0] + 1
        assert cover == L  # intervals partition the grid
        # the candidate grid points contain the exact grid argmin/argmax
        assert full[cands].min() == full.min()
        assert full[cands].max() == full.max()


def test_config_from_reference_yaml_shape():
    from sacenv.config import BoatConfig
    raw = {"base_settings": {"experiment": 6, "test_mode": 1, "dt": 0.25, "t_max": 2500},
           "boat": {"fuel": 30}, "wind": {"max_velocity": 0.5}}
    c = BoatConfig.from_any(raw)
    assert (c.experiment, c.test_mode, c.fuel, c.wind_len) == (6, 1, 30, 10000)

    class Dot(dict):
        __getattr__ = dict.__getitem__
    d = Dot(base_settings=Dot(experiment=2, test_mode=0, dt=0.25, t_max=5))
    c2 = BoatConfig.from_any(d)
    assert (c2.experiment, c2.wind_len) == (2, 20)
    with pytest.raises(ValueError):
        BoatConfig(experiment=7).validate()
    with pytest.raises(ValueError):
        BoatConfig(experiment=6, fixed_points=3).validate()


def test_package_imports_without_gpu():
    import sacenv
    assert sacenv.BoatConfig is not None
    assert "oracle" not in sys.modules.get("sacenv").__dict__


# ---------------------------------------------------------------- replay buffer sampling

def _ring_model(M, S, S2, A, R, D):
    """agent/buffer.py:13-22 store_transition, restated."""
    n = len(R)
    st, st2 = np.zeros((M, S.shape[1])), np.zeros((M, S.shape[1]))
    ac, rw, dn = np.zeros((M, A.shape[1])), np.zeros(M), np.zeros(M, bool)
    for i in range(n):
        j = i % M
        st[j], st2[j], ac[j], rw[j], dn[j] = S[i], S2[i], A[i], R[i], D[i]
    return st, ac, rw, st2, dn


def test_replay_sampling_algorithm_matches_reference():
    """The draw the sampling kernel implements (masked-rejection randint on MT19937
    words, nothing drawn when max_mem == 1) reproduces the reference ReplayBuffer's
    np.random.choice batches and leaves the global stream where numpy does."""
    z = np.load(os.path.join(ROOT, "tests", "golden", "replay_buffer.npz"), allow_pickle=False)
    for c in z["cases"]:
        g = lambda k: z[f"{c}_{k}"]  # noqa: E731
        M, batch, seed = int(g("M")), int(g("batch")), int(g("seed"))
        max_mem = min(len(g("R")), M)
        mt = PyMT(seed)
        idx = np.array([0 if max_mem == 1 else mt.randint(0, max_mem) for _ in range(batch)])
        mem = _ring_model(M, g("S"), g("S2"), g("A"), g("R"), g("D"))
        for got, want in zip((m[idx] for m in mem), ("states", "actions", "rewards", "states_", "dones")):
            np.testing.assert_array_equal(got, g(want), err_msg=f"{c}:{want}")
        # stream state after the draw: the same words consumed as numpy (both twist lazily)
        assert mt.pos == int(g("pos_after")), c
        assert mt.key == [int(x) for x in g("key_after")], c


def test_library_binds_after_torch():
    """_lib.load() imports torch before the CDLL, so the library binds to torch's HIP
    runtime (smoke() loads the library before anything imports torch; bound to
    /opt/rocm's runtime first, its HIP calls found no device on the GPU box)."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, 'sac-agent_amd'); from sacenv import _lib; "
            "assert 'torch' not in sys.modules; _lib.load(); assert 'torch' in sys.modules")
    subprocess.run([sys.executable, "-c", code], check=True, cwd=ROOT)


def _sac_params(**kw):
    from sacenv import _lib
    base = dict(obs_dim=11, n_actions=1, hidden=256, batch=1024, max_action=1.0, gamma=0.99, tau=0.005,
                reward_scale=10.0, lr_actor=0.005, lr_critic=3e-4, adam_beta1=0.9, adam_beta2=0.999,
                adam_eps=1e-8)
    base.update(kw)
    return _lib.SacParams(**base)


def test_sac_layout(built_lib):
    """The SAC weights buffer: torch-shaped tensors per net, 16-B aligned and disjoint,
    Adam states and transposes after the five nets, scratch sized for the batch."""
    from sacenv import _lib
    L = _lib.sac_layout(_sac_params())
    H, D = 256, 11
    sizes = {0: [(H * D), H, H * H, H, H, 1, H, 1], 1: [H * (D + 1), H, H * H, H, H, 1, -1, -1],
             2: [H * D, H, H * H, H, H, 1, -1, -1]}
    for s in range(3):
        spans = []
        for k, n in enumerate(sizes[s]):
            off = L.tensor[s][k]
            if n < 0:
                assert off == -1
                continue
            assert off % 4 == 0
            spans.append((off, off + n))
        spans.sort()
        for (a0, a1), (b0, b1) in zip(spans, spans[1:]):
            assert a1 <= b0
        assert spans[-1][1] <= L.net_floats[s]
    shapes = [0, 1, 1, 2, 2]
    regions = [(L.net[n], L.net[n] + L.net_floats[shapes[n]]) for n in range(5)]
    regions += [(L.adam_m[n], L.adam_m[n] + L.net_floats[shapes[n]]) for n in range(4)]
    regions += [(L.adam_v[n], L.adam_v[n] + L.net_floats[shapes[n]]) for n in range(4)]
    regions += [(L.w2f[n], L.w2f[n] + H * H) for n in range(5)]
    regions += [(L.w2tf[n], L.w2tf[n] + H * H) for n in range(4)]
    regions.sort()
    for (a0, a1), (b0, b1) in zip(regions, regions[1:]):
        assert a1 <= b0 and a0 % 4 == 0
    assert regions[-1][1] == L.total_floats
    assert L.scratch_bytes == 4 * 1024 * (16 * H + 27 + 16)  # activations, 27 row fields, X^T


def test_sac_argument_errors_without_gpu(built_lib):
    import ctypes
    from sacenv import _lib
    lay = _lib.SacLayout()
    assert built_lib.sacenv_sac_layout(ctypes.byref(_sac_params(batch=1000)), ctypes.byref(lay)) == -4
    assert built_lib.sacenv_sac_layout(ctypes.byref(_sac_params(hidden=128)), ctypes.byref(lay)) == -4
    assert built_lib.sacenv_sac_layout(ctypes.byref(_sac_params(n_actions=2)), ctypes.byref(lay)) == -4
    assert built_lib.sacenv_sac_layout(ctypes.byref(_sac_params(obs_dim=15)), ctypes.byref(lay)) == -4
    assert built_lib.sacenv_sac_layout(None, ctypes.byref(lay)) == -1
    p = _sac_params()
    args = [None] * 9
    assert built_lib.sacenv_sac_learn(ctypes.byref(p), *args, 1, None, None) == -1
    assert built_lib.sacenv_sac_learn(ctypes.byref(p), *([16] * 9), 0, None, None) == -5
    assert built_lib.sacenv_sac_learn(ctypes.byref(p), *([8] * 9), 1, None, None) == -4  # unaligned
    assert built_lib.sacenv_sac_act(ctypes.byref(p), None, None, 4, None, None, None, None) == -1
    assert built_lib.sacenv_sac_act(ctypes.byref(p), None, None, 0, None, None, None, None) == 0


def test_native_sac_has_no_cpu_path(built_lib):
    """NativeSAC runs on the SAC kernels only: a CPU device is refused, not emulated."""
    from sacenv import _lib
    from sacenv.sac_native import NativeSAC
    with pytest.raises(_lib.SacenvError):
        NativeSAC("cpu", init_seed=0, with_memory=False)


def test_native_sac_views_follow_the_c_layout(built_lib):
    """The torch parameter views NativeSAC builds sit at the C layout's tensor offsets."""
    from sacenv import _lib
    L = _lib.sac_layout(_sac_params())
    # actor: w1 [256][11] at tensor[0][0]; critic w1 [256][12]; value heads follow fc2.bias
    assert L.tensor[0][2] - L.tensor[0][0] == 256 * 11 + 256  # 2 816 floats of fc1.weight are 16-B aligned
    assert L.tensor[1][1] == 256 * 12 and L.tensor[2][6] == -1 and L.tensor[0][6] > L.tensor[0][5]


def test_closed_loop_co_residency_plan_arithmetic():
    """sacenv.closed_loop's plan (no GPU): every owner wave resident with room for one
    policy wave per SIMD (512 VGPRs, granule 8) and one padded policy workgroup per CU."""
    from sacenv import _lib
    from sacenv.closed_loop import make_plan
    p = make_plan(256, 1024, 318, 2816, 1024, 150, 84 * 1024, 65536)   # the measured kernels
    assert p.seg_vgprs == 320 and p.act_vgprs == 152 and p.owner_waves_per_simd == 1
    assert p.max_envs == 65536
    with pytest.raises(ValueError):
        make_plan(256, 1025, 318, 2816, 1025, 150, 84 * 1024, 65600)      # one owner wave more
    with pytest.raises(ValueError):
        make_plan(256, 2048, 318, 2816, 2048, 150, 84 * 1024, 131072)     # two per SIMD
    assert make_plan(256, 2048, 176, 2816, 2048, 150, 84 * 1024).max_envs == 131072  # 2 x 176 + 152
    with pytest.raises(_lib.SacenvError):
        make_plan(256, 64, 318, 2816, 64, 150, 80 * 1024)                 # 2 policy WGs would fit a CU
    with pytest.raises(ValueError):                                      # LDS: owners + one policy WG
        make_plan(256, 1024, 100, 40 * 1024, 1024, 150, 84 * 1024)
