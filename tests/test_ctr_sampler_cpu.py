"""The staged replay's counter-based sampler, on the CPU: the oracle's Philox4x64-10
against numpy's own C implementation (np.random.Philox), the draw rule's range, skip
and uniformity, and the all-gather chunk's capacity rule (sacenv_replay_stage_chunk,
host code in libsacenv.so: no GPU call) against simulated per-rank counts.

Reference: agent/buffer.py:24-35 (np.random.choice(max_mem, batch) with
max_mem = min(mem_cntr, mem_size)), agent/continuous_agent.py:97-98 (learn()
returns while fewer than batch rows are stored).
"""
import ctypes as C

import numpy as np
import pytest

import ctr_sampler as cs


@pytest.mark.parametrize("seed", [0, 1, 5, 2**32 - 1, 2**64 - 1, 0x0123456789ABCDEF])
def test_philox_matches_numpy(seed):
    ctrs = [(0, 0, 0, 0), (1, 0, 0, 0), (1023, 255, 0, 0), (2**64 - 1, 0, 0, 0), (2**64 - 1, 2**64 - 1, 3, 0),
            (7, 123456789, 1, 0), (0, 0, 0, 1)]
    got = cs.philox4x64_10(np.array(ctrs, dtype=np.uint64), seed, 0)
    for c, row in zip(ctrs, got):
        assert np.array_equal(row, cs.numpy_philox_block(seed, c)), (seed, c)


def test_draw_rule_is_the_first_accepted_word():
    """draw i takes word i % 4 of the blocks at counters (i // 4, L, j, 0), j = 0, 1, ...:
    the first accepted one (a range with a 50 % rejection rate exercises the retries)."""
    for seed, L, B, period, M in ((9, 40, 64, 1000, 30_011), (3, 2, 200, 1000, 1025)):
        idx = cs.draw_learn(seed, L, B, period, M)
        rng = min((L + 1) * period, M) - 1
        mask = cs.range_mask(rng)
        retried = 0
        for i in range(B):
            for j in range(64):
                w = int(cs.philox4x64_10(np.array([[i // 4, L, j, 0]], np.uint64), seed, 0)[0][i % 4]) & mask
                if w <= rng:
                    assert idx[i] == w, (seed, i, j)
                    retried += j > 0
                    break
        if M == 1025:
            assert retried > 20


def test_draw_range_and_skip_rule():
    B, period, M = 700, 300, 19_000
    for L in range(8):
        idx = cs.draw_learn(3, L, B, period, M)
        c = (L + 1) * period
        if c < B:
            assert (idx == -1).all()
        else:
            assert idx.min() >= 0 and idx.max() < min(c, M)
    assert (cs.draw_learn(3, 0, 1, 1, 10) == 0).all()    # one row stored: np.random.choice(1, 1) = 0


def test_draws_are_uniform_and_independent_of_neighbours():
    # 64 learns x 4 096 draws over 1 000 rows (mask 1023: 2.4 % rejected words)
    idx = np.concatenate([cs.draw_learn(11, L, 4096, 5000, 1000) for L in range(64)])
    counts = np.bincount(idx, minlength=1000)
    exp = idx.size / 1000
    chi2 = ((counts - exp) ** 2 / exp).sum()
    assert chi2 < 1000 + 6 * np.sqrt(2 * 1000), chi2        # dof 999
    a, b = cs.draw_learn(11, 5, 4096, 5000, 1000), cs.draw_learn(11, 6, 4096, 5000, 1000)
    assert (a == b).mean() < 0.01                           # learns are not copies of each other


def _chunk(lib, n, world, M, B, seg):
    from sacenv import _lib
    p = _lib.ReplayParams()
    p.mem_size, p.obs_dim, p.act_dim, p.reward_f32, p.terminal_mask = M, 11, 1, 1, 2
    sp = _lib.StagedParams()
    sp.period, sp.offset, sp.n, sp.n_pad, sp.seg, sp.experiment = world * n, 0, n, -(-n // 64) * 64, seg, 6
    cap, nbytes = C.c_int64(), C.c_int64()
    assert lib.sacenv_replay_stage_chunk(C.byref(p), C.byref(sp), B, seg, C.byref(cap), C.byref(nbytes)) == 0
    return cap.value, nbytes.value


def _owner_counts(n, world, M, B, seg, g, seed=1):
    """Records each rank packs for segment g (rank 0: + the skipped learns' rows)."""
    period = world * n
    cnt = np.zeros(world, np.int64)
    for k in range(seg):
        L = g * seg + k
        c = (L + 1) * period
        idx = cs.draw_learn(seed, L, B, period, M)
        if c < B:
            cnt[0] += B
            continue
        s = idx + M * ((c - 1 - idx) // M)
        cnt += np.bincount((s % period) // n, minlength=world)
    return cnt


@pytest.mark.parametrize("n,world,M,B,seg", [(1000, 2, 30_011, 333, 32), (700, 4, 50_000, 256, 32),
                                             (65_536, 8, 1_000_000, 64, 16), (300, 3, 19_000, 700, 64)])
def test_chunk_capacity_covers_every_rank(built_lib, n, world, M, B, seg):
    cap, nbytes = _chunk(built_lib, n, world, M, B, seg)
    assert nbytes >= 16 + 100 * cap and nbytes % 256 == 0
    worst = max(_owner_counts(n, world, M, B, seg, g).max() for g in range(3))
    assert worst <= cap <= B * seg
    # the chunk is close to a rank's share, not the whole batch (the all-gather's point)
    if B * seg >= 4096 and -(-B // n) <= 1:
        assert cap < 1.6 * B * seg / world + 8 * np.sqrt(B * seg) + 64, (cap, B * seg / world)


def test_chunk_at_the_bench_shape(built_lib):
    """65 536 envs per rank, ReplayBuffer(10^6), batch 1 024, 256-step segments: each
    rank's chunk at N = 8 is ~13 % of the slots (the ring window holds two steps of
    the last ranks' envs), so an all-gather sends ~25 MB per rank against the ring
    all-reduce's 2 x 7/8 x 27.3 MB."""
    cap, nbytes = _chunk(built_lib, 65_536, 8, 1_000_000, 1024, 256)
    total = 1024 * 256
    assert 0.13 * total < cap < 0.14 * total
    allgather_send = 7 * nbytes
    allreduce_send = 2 * 7 / 8 * total * 26 * 4
    assert allgather_send < 0.56 * allreduce_send
    cap1, _ = _chunk(built_lib, 65_536, 1, 1_000_000, 1024, 256)
    assert cap1 == total
