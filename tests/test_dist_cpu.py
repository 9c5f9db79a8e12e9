"""World-size 1/2/4 gloo tests of the env-parallel record gather (CPU, no GPU).

Each rank runs its shard of envs (global-id seeds) on the CPU oracle, packs
the step outputs in the kernel's record layout and all-gathers them; rank 0
checks the pooled records equal a single-process run over all envs, i.e.
results are independent of the world size.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT

N_PER_RANK, STEPS = 6, 40


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    for p in (os.path.join(ROOT, "sac-agent_amd"), os.path.join(ROOT, "oracle")):
        sys.path.insert(0, p)
    from boat_oracle import OracleConfig, OracleVecBoat
    from sacenv.dist import RecordLayout, gather_records, shard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        off, n = shard(rank, world, N_PER_RANK)
        seeds = np.arange(off, off + n, dtype=np.uint64) + 100
        ora = OracleVecBoat(OracleConfig(experiment=6), seeds, max_episode_steps=25)
        ora.reset()
        lay = RecordLayout(n)
        acts = np.random.default_rng(0).uniform(-1, 1, (STEPS, world * N_PER_RANK)).astype(np.float32)
        pooled = []
        for k in range(STEPS):
            r = ora.step(acts[k, off:off + n])
            rec = lay.pack(torch.from_numpy(r["reset_obs"]), torch.from_numpy(r["reward"]),
                           torch.from_numpy(r["done"]), torch.from_numpy(r["term"]))
            g = gather_records(rec)
            pooled.append([t.numpy().copy() for t in lay.unpack_gathered(g, world)])
        if rank == 0:
            q.put(pooled)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2, 4])
def test_gather_pools_all_shards(world):
    """gloo at world sizes 1-4."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from boat_oracle import OracleConfig, OracleVecBoat
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    pooled = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    # single-process reference over all global envs
    seeds = np.arange(world * N_PER_RANK, dtype=np.uint64) + 100
    ora = OracleVecBoat(OracleConfig(experiment=6), seeds, max_episode_steps=25)
    ora.reset()
    acts = np.random.default_rng(0).uniform(-1, 1, (STEPS, world * N_PER_RANK)).astype(np.float32)
    for k in range(STEPS):
        r = ora.step(acts[k])
        obs, rew, done, term = pooled[k]
        np.testing.assert_array_equal(obs, r["reset_obs"].astype(np.float32))
        np.testing.assert_array_equal(rew, r["reward"].astype(np.float32))
        np.testing.assert_array_equal(done, r["done"])
        np.testing.assert_array_equal(term, r["term"])


def test_record_layout_roundtrip():
    import sys
    sys.path.insert(0, os.path.join(ROOT, "sac-agent_amd"))
    from sacenv.dist import RecordLayout
    lay = RecordLayout(5)
    obs = torch.arange(55, dtype=torch.float32).view(5, 11)
    rec = lay.pack(obs, torch.ones(5), torch.tensor([0, 1, 0, 0, 1]), torch.tensor([0, 4, 0, 0, 6]))
    assert rec.numel() == 250
    o, r, d, t = lay.views(rec)
    assert torch.equal(o, obs) and d.tolist() == [0, 1, 0, 0, 1] and t.tolist() == [0, 4, 0, 0, 6]
    with pytest.raises(ValueError):
        lay.views(torch.zeros(10, dtype=torch.uint8))


def _seg_worker(rank, world, port, seg, q):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "sac-agent_amd"))
    from sacenv.dist import SegmentPool, gather_records
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rb = 50 * 3
        pool = SegmentPool(rb, seg, "cpu")
        rng = np.random.default_rng(rank)
        per_step, pooled = [], []
        for k in range(STEPS):
            rec = torch.from_numpy(rng.integers(0, 256, rb, dtype=np.uint8))
            per_step.append(gather_records(rec.clone()))
            pool.push([rec[:100], rec[100:]])  # two record parts fill one row
            if pool.last is not None:
                out, n = pool.last
                pooled += [pool.step_records(out, n, j) for j in range(n)]
                pool.last = None
        out = pool.flush()  # the partial last segment
        if out is not None:
            n = pool.last[1]
            pooled += [pool.step_records(out, n, j) for j in range(n)]
        ok = len(pooled) == STEPS and all(torch.equal(a, b) for a, b in zip(pooled, per_step))
        q.put((rank, ok, pool.flushes))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,seg", [(2, 8), (2, 7), (3, 16)])
def test_segment_pool_equals_per_step_gathers(world, seg):
    """SegmentPool (one all-gather per segment, as bench.py at N>1) pools the
    same per-step records as one all-gather per step, partial segments too."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_seg_worker, args=(r, world, port, seg, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert all(ok for _, ok, _ in res), res
    assert all(f == -(-STEPS // seg) for _, _, f in res), res


def _transition_worker(rank, world, port, seg, q):
    import sys
    for p in (os.path.join(ROOT, "sac-agent_amd"), os.path.join(ROOT, "oracle")):
        sys.path.insert(0, p)
    from boat_oracle import OracleConfig, OracleVecBoat
    from sacenv.config import BoatConfig, first_obs_template
    from sacenv.dist import SegmentPool, TransitionLayout, TransitionStream, shard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        off, n = shard(rank, world, N_PER_RANK)
        seeds = np.arange(off, off + n, dtype=np.uint64) + 100
        # a short track and truncation: envs end (OOB, rudder, truncation) every few steps
        ora = OracleVecBoat(OracleConfig(experiment=6, track_width=60.0), seeds, max_episode_steps=9)
        reset_obs = torch.from_numpy(ora.reset()).to(torch.float32)
        lay = TransitionLayout(n, 64)     # the kernel pads rows to 64
        pool = SegmentPool(lay.nbytes, seg, "cpu")
        g_reset = torch.empty(world * n, 11)
        dist.all_gather(list(g_reset.chunk(world)), reset_obs)
        first = torch.from_numpy(first_obs_template(BoatConfig.from_any({"boat_env": {"track_width": 60}})))
        stream = TransitionStream(lay, world, g_reset, first)
        acts = np.random.default_rng(0).uniform(-1, 1, (STEPS, world * N_PER_RANK)).astype(np.float32)
        out = []

        def drain():
            if pool.last is not None:
                g, m = pool.last
                out.extend(stream.push(pool.step_records(g, m, j)) for j in range(m))
                pool.last = None

        for k in range(STEPS):
            r = ora.step(acts[k, off:off + n])
            t = lambda x: torch.from_numpy(np.asarray(x))  # noqa: E731
            # what sacenv_boat_step_pooled writes: s' before the reset, and the new
            # episode's obs[3] where an env restarted
            row = lay.pack(t(r["obs"]), t(r["reward"]), t(acts[k, off:off + n]),
                           t(r["reset_obs"][:, 3]), t(r["term"]))
            pool.push([row])
            drain()
        pool.flush()
        drain()
        if rank == 0:
            q.put([[x.numpy().copy() for x in tr] for tr in out])
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,seg", [(2, 8), (2, 5)])
def test_pooled_transitions_equal_single_process(world, seg):
    """N>1 pooling carries whole transitions (main.py:83-88, buffer.py:13-22): the
    pooled (s, a, r, s', code) of every global env equal a single-process run,
    including envs that ended (s' = the terminal obs, and the next s = the new
    episode's first obs rebuilt from the fresh-Boat template + obs3_next)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from boat_oracle import OracleConfig, OracleVecBoat
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_transition_worker, args=(r, world, port, seg, q)) for r in range(world)]
    for p in procs:
        p.start()
    pooled = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert len(pooled) == STEPS
    seeds = np.arange(world * N_PER_RANK, dtype=np.uint64) + 100
    ora = OracleVecBoat(OracleConfig(experiment=6, track_width=60.0), seeds, max_episode_steps=9)
    s = ora.reset().astype(np.float32)
    acts = np.random.default_rng(0).uniform(-1, 1, (STEPS, world * N_PER_RANK)).astype(np.float32)
    ended = 0
    for k in range(STEPS):
        r = ora.step(acts[k])
        ps, pa, pr, pn, pc = pooled[k]
        # entries 0..8 travel in the row (bit-exact); 9 (rudder) and 10 (fuel) are rebuilt
        # in the kernel's arithmetic, the oracle divides: equal to an f32 ulp
        np.testing.assert_array_equal(ps[:, :9], s[:, :9])
        np.testing.assert_allclose(ps[:, 9:], s[:, 9:], rtol=2e-7, atol=0)
        np.testing.assert_array_equal(pa, acts[k])
        np.testing.assert_array_equal(pr, r["reward"].astype(np.float32))
        want = r["obs"].astype(np.float32)  # terminal obs where done
        np.testing.assert_array_equal(pn[:, :9], want[:, :9])
        np.testing.assert_allclose(pn[:, 9:], want[:, 9:], rtol=2e-7, atol=0)
        np.testing.assert_array_equal(pc, r["term"])
        ended += int(r["done"].sum())
        s = r["reset_obs"].astype(np.float32)
    assert ended > STEPS // 2   # the ended-env rows were exercised


def _sharded_worker(rank, world, port, n, M, steps, B, q):
    """Rank-local ring rows (this rank's transitions only, at the pooled buffer's
    positions), shared sampling stream, integer SUM all-reduce of the owned rows."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "sac-agent_amd"))
    from sacenv.dist import shard_owner
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        W = world * n
        ring = np.zeros((M, 3), np.int64)          # a row's payload: (step, global env, marker)
        rs = np.random.RandomState(11)             # every rank: the same stream
        cntr, out = 0, []
        for t in range(steps):
            rows = (cntr + rank * n + np.arange(n)) % M   # sacenv_replay_store_shard's positions
            ring[rows] = np.stack([np.full(n, t), rank * n + np.arange(n), np.full(n, 7)], 1)
            cntr += W
            if t % 2 == 1:
                idx = rs.choice(min(cntr, M), B)   # buffer.py:27
                own = shard_owner(idx, cntr, M, W, n) == rank
                mine = torch.from_numpy(np.where(own[:, None], ring[idx], 0))
                dist.all_reduce(mine, op=dist.ReduceOp.SUM)
                out.append((idx, mine.numpy()))
        q.put((rank, out))
    except Exception as exc:  # noqa: BLE001
        q.put((rank, repr(exc)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n,M", [(2, 5, 23), (3, 4, 50), (2, 8, 16)])
def test_sharded_replay_equals_pooled_buffer(world, n, M):
    """SURVEY §8(e)'s lighter exchange, on gloo: each rank writes only its own rows
    (at the pooled ring's positions), every rank draws the same indices, and one SUM
    all-reduce of the owned rows gives the pooled buffer's batch -- including rows
    that wrapped around the ring and changed writer (M not a multiple of world * n)."""
    steps, B = 12, 9
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_sharded_worker, args=(r, world, port, n, M, steps, B, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert all(not isinstance(v, str) for v in res.values()), res
    # the pooled buffer: one process stores every rank's rows in global env order
    W = world * n
    ring = np.zeros((M, 3), np.int64)
    rs = np.random.RandomState(11)
    cntr, k = 0, 0
    for t in range(steps):
        ring[(cntr + np.arange(W)) % M] = np.stack([np.full(W, t), np.arange(W), np.full(W, 7)], 1)
        cntr += W
        if t % 2 == 1:
            idx = rs.choice(min(cntr, M), B)
            for r in range(world):
                got_idx, got = res[r][k]
                np.testing.assert_array_equal(got_idx, idx)
                np.testing.assert_array_equal(got, ring[idx])
            k += 1
