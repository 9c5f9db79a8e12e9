"""Oracle (TEST INFRASTRUCTURE ONLY -- never imported by the product path) of the
staged replay's counter-based sampler (sacenv_replay_stage_draw_ctr,
sac-agent_amd/csrc/sacenv_replay.hip k_rb_draw_ctr).

What it restates. The reference's learn() samples ``np.random.choice(max_mem,
batch)`` (agent/buffer.py:27; max_mem = min(mem_cntr, mem_size), buffer.py:26),
i.e. `batch` ring rows uniform with replacement, and skips the learn while fewer
than `batch` rows are stored (agent/continuous_agent.py:97-98). The counter-based
sampler keeps that distribution and that skip rule but takes its words from
Philox4x64-10 instead of the one MT19937 stream: draw i of global learn L (after
L + 1 pooled steps, c = (L + 1) x period rows stored) takes word i mod 4 of the
Philox4x64-10 blocks at counters (i div 4, L, j, 0), key (seed, 0), j = 0, 1, ...:
the first whose bits under numpy's mask (the smallest 2^b - 1 >= range - 1) are
<= range - 1 -- the masked rejection numpy's legacy bounded draw applies to MT words
(numpy/random/src/distributions: random_bounded_uint64 with use_masked). One block
serves four draws (the device draws a segment with a quarter of the Philox work).

Pinning. ``philox4x64_10`` is this file's own restatement of the published
generator (Salmon, Moraes, Dror, Shaw, "Parallel random numbers: as easy as 1,
2, 3", SC'11: multipliers 0xD2E7470EE14C6C93 / 0xCA5A826395121157, Weyl key
increments 0x9E3779B97F4A7C15 / 0xBB67AE8584CAA73B, 10 rounds);
tests/test_ctr_sampler_cpu.py checks it word for word against numpy's C
implementation, ``np.random.Philox`` (numpy 2.2 in this image: its random_raw()
after ``counter=c`` returns the four words of the block at counter c + 1), and the
draw rule's range / skip / uniformity properties.
"""
from __future__ import annotations

import numpy as np

M0 = np.uint64(0xD2E7470EE14C6C93)
M1 = np.uint64(0xCA5A826395121157)
W0 = np.uint64(0x9E3779B97F4A7C15)
W1 = np.uint64(0xBB67AE8584CAA73B)
_LO = np.uint64(0xFFFFFFFF)
_S32 = np.uint64(32)


def _mulhilo(a: np.uint64, b: np.ndarray):
    """(hi, lo) of the 128-bit products a * b, elementwise (uint64 arrays)."""
    a_lo, a_hi = a & _LO, a >> _S32
    b_lo, b_hi = b & _LO, b >> _S32
    ll = a_lo * b_lo
    lh = a_lo * b_hi
    hl = a_hi * b_lo
    hh = a_hi * b_hi
    mid = (ll >> _S32) + (lh & _LO) + (hl & _LO)
    hi = hh + (lh >> _S32) + (hl >> _S32) + (mid >> _S32)
    lo = a * b
    return hi, lo


def philox4x64_10(ctr: np.ndarray, key0, key1) -> np.ndarray:
    """Philox4x64-10 of counters ctr [n, 4] (uint64) under key (key0, key1): [n, 4]."""
    c = np.array(ctr, dtype=np.uint64).reshape(-1, 4).copy()
    k0 = np.uint64(key0)
    k1 = np.uint64(key1)
    with np.errstate(over="ignore"):
        for _ in range(10):
            hi0, lo0 = _mulhilo(M0, c[:, 0])
            hi1, lo1 = _mulhilo(M1, c[:, 2])
            c = np.stack([hi1 ^ c[:, 1] ^ k0, lo1, hi0 ^ c[:, 3] ^ k1, lo0], axis=1)
            k0 = k0 + W0
            k1 = k1 + W1
    return c


def range_mask(rng: int) -> int:
    m = int(rng)
    for s in (1, 2, 4, 8, 16, 32):
        m |= m >> s
    return m


def draw_learn(seed: int, L: int, batch: int, period: int, mem_size: int) -> np.ndarray:
    """idx [batch] of global learn L (k_rb_draw_ctr): -1 when the learn is skipped."""
    c = (L + 1) * period
    if c < batch:
        return np.full(batch, -1, np.int64)
    rng = min(c, mem_size) - 1
    if rng == 0:
        return np.zeros(batch, np.int64)
    mask = np.uint64(range_mask(rng))
    out = np.full(batch, -1, np.int64)
    todo = np.arange(batch, dtype=np.int64)
    for j in range(64):
        ctr = np.zeros((todo.size, 4), np.uint64)
        ctr[:, 0] = (todo // 4).astype(np.uint64)
        ctr[:, 1] = np.uint64(L)
        ctr[:, 2] = np.uint64(j)
        words = philox4x64_10(ctr, np.uint64(seed), np.uint64(0))[np.arange(todo.size), todo % 4] & mask
        hit = words <= np.uint64(rng)
        out[todo[hit]] = words[hit].astype(np.int64)
        todo = todo[~hit]
        if todo.size == 0:
            break
    out[todo] = 0   # (64 rejected words in a row: probability < 2^-64; the device's bound)
    return out


def draw_segment(seed: int, g: int, seg: int, batch: int, period: int, mem_size: int) -> np.ndarray:
    """idx [seg, batch] of segment g's learns (global learns g*seg .. g*seg + seg - 1)."""
    return np.stack([draw_learn(seed, g * seg + k, batch, period, mem_size) for k in range(seg)])


def numpy_philox_block(seed: int, ctr: tuple[int, int, int, int]) -> np.ndarray:
    """The block numpy's own Philox generator produces at counter ``ctr`` (key (seed, 0)):
    random_raw() after counter = ctr - 1 (numpy increments before it generates)."""
    c = ctr[0] | (ctr[1] << 64) | (ctr[2] << 128) | (ctr[3] << 192)
    bg = np.random.Philox(key=int(seed), counter=(c - 1) % (1 << 256))
    return np.asarray(bg.random_raw(4), dtype=np.uint64)
