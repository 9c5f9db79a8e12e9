"""StagedReplay: the pooled replay buffer sampled out of staged segments.

The reference loop (main.py:78-90) stores every env's transition (buffer.py:13-22)
and runs one learn() -- sample_buffer(batch), buffer.py:24-35 -- after EVERY step,
each on the buffer as that step left it. StagedReplay draws a segment's learns
after the segment from the rows the persistent launch wrote
(sacenv_boat_segment's ``stage``), with no ring. The learns' index draws are
made ahead (they depend only on the sampling stream and the stored counts), and
the launch writes only the rows those learns read. The reference side here is the
literal loop on the device: a VecBoatEnv stepped one launch at a time, a
DeviceReplayBuffer fed every step (store_env_step: the reference's persistent
terminal rule, new_state = the terminal obs of envs that reset) and sampled
after every step. Batches and indices must agree bit for bit, across the ring's
wrap (mem_size not a multiple of the rows per step), ranges below mem_size at
the start, learns skipped while fewer rows than a batch are stored, auto-resets
(experiment 2's start-y obs entry included) and, over two gloo ranks sharing the
box's GPU, the SUM all-reduce of the ranks' shares.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT

pytestmark = pytest.mark.gpu

SEG = 64


_BITS = torch.tensor([bin(i).count("1") for i in range(256)], dtype=torch.int64)


def _popcount(t: torch.Tensor) -> int:
    return int(_BITS.to(t.device)[t.view(torch.uint8).long()].sum())


def _cfg(exp):
    return {"base_settings": {"experiment": exp, "test_mode": 0}, "boat_env": {"track_width": 30}}


def _run(rank, world, exp, N, M, B, n_segs, dev, group=None, sampler="mt", exchange="allreduce", fused=False,
         emulate=False):
    """Returns (n learns checked, n skipped) on rank 0 (None elsewhere).

    sampler "mt": the indices equal the reference stream's (DeviceReplayBuffer.sample
    after every step). sampler "philox": the indices equal the CPU oracle's
    counter-based draws (oracle/ctr_sampler.py, pinned to numpy's Philox), lie in
    [0, min(cntr, M)), and the batch equals DeviceReplayBuffer.gather of the same
    indices from the buffer fed every step. fused (philox + allgather): each
    segment's side work is ONE launch (side_segment: the unpack of the segment
    before, the pack of this one, the draws of the one after next), as
    SegmentExchange runs it. emulate (rank 0 of `world`, one process): the collective
    stood in for and the other ranks' chunks packed from this GPU's rows (timing
    only), so only the slots this rank owns are compared."""
    from sacenv import VecBoatEnv
    from sacenv.replay import DeviceReplayBuffer, StagedReplay
    import ctr_sampler
    kw = dict(seed=3, device=dev, max_episode_steps=40, n_helpers=64, auto_refill=False)
    env = VecBoatEnv(_cfg(exp), N, env_id_offset=rank * N, **kw)
    obs0 = env.reset().clone()
    rep = StagedReplay(N, env.n_pad, exp, env.first_obs_template(), rank=rank, world=world, mem_size=M,
                       batch=B, seg=SEG, seed=5, device=dev, group=group, sampler=sampler, exchange=exchange,
                       standin=dict(bytes=0, workgroups=4, us=1.0) if emulate else None)
    assert rep.emulated == emulate
    assert rep.fused == (sampler == "philox" and exchange == "allgather")
    rep.begin(obs0)
    assert bool((env.last_term == 0).all())
    ref = ref_rb = None
    if rank == 0:
        ref = VecBoatEnv(_cfg(exp), world * N, **kw)
        ref.reset()
        ref_rb = DeviceReplayBuffer(M, (11,), 1, device=dev, seed=5)
    g = torch.Generator(device=dev)
    g.manual_seed(9)
    written = 0
    acts_all, gots = [], []
    for s in range(n_segs):
        acts = torch.rand((SEG, world * N), generator=g, device=dev) * 2 - 1
        acts_all.append(acts)
        mine = acts[:, rank * N:(rank + 1) * N].contiguous()
        sa = rep.stage_args(s)
        written += _popcount(sa["marks"])   # (complete before the launch, which consumes them)
        env.segment_async(mine, SEG, stage=sa["stage"], stage_marks=sa["marks"])
        env.refill()
        if fused:
            got = rep.side_segment(s, s - 1 if s > 0 else None)
            rep.collect_segment(s)
            if got is not None:
                gots.append([tuple(x.clone() for x in b) for b in got])
        else:
            rep.prepare(s + 1)
            gots.append([tuple(x.clone() for x in b) for b in rep.sample_segment(s)])
        assert _popcount(rep.stage_args(s)["marks"]) == 0   # the launch cleared the marks it read
    if fused:
        gots.append([tuple(x.clone() for x in b) for b in rep.unpack_segment(n_segs - 1)])
    checked = skipped = 0
    for s in range(n_segs if ref is not None else 0):
        acts, got = acts_all[s], gots[s]
        for k in range(SEG):
            prev = ref.obs.clone()
            ref.step(acts[k].contiguous())
            ref_rb.store_env_step(prev, acts[k].contiguous(), ref)
            st, ac, rw, ns, tm, idx = got[k]
            if ref_rb.mem_cntr < B:     # continuous_agent.learn returns before sampling
                torch.cuda.synchronize()
                assert bool((idx == -1).all()) and not bool(st.any()), (s, k)
                skipped += 1
                continue
            if sampler == "mt":
                want = ref_rb.sample(B)
                torch.cuda.synchronize()
                assert torch.equal(idx, want[5]), f"segment {s} learn {k}: indices"
            else:
                drawn = ctr_sampler.draw_learn(5, s * SEG + k, B, world * N, M)
                assert torch.equal(idx.cpu(), torch.from_numpy(drawn)), f"segment {s} learn {k}: indices"
                assert int(idx.min()) >= 0 and int(idx.max()) < min(ref_rb.mem_cntr, M)
                want = ref_rb.gather(idx)
                torch.cuda.synchronize()
            own = slice(None)
            if emulate and s > 0:   # (the other ranks' chunks are segment 0's: their records would
                checked += 1        # overwrite this rank's slots of later segments; timing only)
                continue
            if emulate:   # the slots whose row lies in this rank's envs (ring row -> sequence -> env)
                cntr = (s * SEG + k + 1) * world * N
                row = idx.cpu().numpy()
                seq = row + M * ((cntr - 1 - row) // M)
                own = torch.from_numpy(seq % (world * N) < N).to(dev)
                assert 0 < int(own.sum()) < B
            for i, (x, y) in enumerate(zip((st, ac, rw, ns, tm), want[:5])):
                x, y = x.reshape(B, -1)[own], y.reshape(B, -1).to(x.dtype)[own]
                assert torch.equal(x, y), (s, k, i)
            checked += 1
        ref.refill()
        torch.cuda.synchronize()
        # the arena carries info['termination'] as the buffer's per-env byte does
        assert torch.equal(ref.last_term.to(torch.uint8), ref_rb._last_term[ref]), s
    torch.cuda.synchronize()
    env.check_status()
    rep.check()
    if rank == 0 and world == 1:
        # only the rows a learn reads (and their predecessors) were written: at most
        # 2 x 2 marks per sampled row of two segments' learns
        assert 0 < written <= min(n_segs * SEG * N, 4 * n_segs * SEG * B), written
        if 4 * B < N // 2:
            assert written < 0.5 * n_segs * SEG * N, written
    return (checked, skipped) if rank == 0 else None


@pytest.mark.parametrize("exp,N,M,B", [(6, 3000, 50_021, 256), (2, 2000, 40_000, 511), (6, 700, 20_000, 1024),
                                       (5, 1500, 30_011, 300), (1, 1100, 25_000, 128)])
def test_staged_replay_equals_per_step_learns(exp, N, M, B, gpu, built_lib):
    checked, skipped = _run(0, 1, exp, N, M, B, 4, gpu)
    assert checked + skipped == 4 * SEG
    assert skipped == (1 if N < B else 0)


@pytest.mark.parametrize("sampler,exchange,exp,N,M,B", [
    ("philox", "allgather", 6, 3000, 50_021, 256), ("philox", "allgather", 2, 2000, 40_000, 511),
    ("philox", "allgather", 6, 700, 20_000, 1024), ("philox", "allreduce", 5, 1500, 30_011, 300),
    ("mt", "allgather", 6, 3000, 50_021, 256), ("philox", "allgather", 1, 300, 19_000, 700)])
def test_staged_replay_counter_sampler_and_allgather(sampler, exchange, exp, N, M, B, gpu, built_lib):
    """The counter-based sampler (range, skip rule, rows and terminals assembled as the
    buffer fed every step holds them at the same indices) and the packed all-gather
    exchange (at world 1: pack + unpack) against the literal loop."""
    checked, skipped = _run(0, 1, exp, N, M, B, 4, gpu, sampler=sampler, exchange=exchange)
    assert checked + skipped == 4 * SEG
    assert skipped == -(-B // N) - 1  # learns while fewer than B rows are stored


@pytest.mark.parametrize("exp,N,M,B", [(6, 3000, 50_021, 256), (2, 2000, 40_000, 511), (6, 700, 20_000, 1024)])
def test_staged_replay_side_launch(exp, N, M, B, gpu, built_lib):
    """The fused side launch (sacenv_replay_stage_side: unpack g - 1, pack g, draw g + 2 in
    one launch) against the literal loop, as the separate calls are."""
    checked, skipped = _run(0, 1, exp, N, M, B, 5, gpu, sampler="philox", exchange="allgather", fused=True)
    assert checked + skipped == 5 * SEG
    assert skipped == -(-B // N) - 1


def test_staged_replay_emulated_rank_of_four(gpu, built_lib):
    """bench.py's replay_path_rank_of_W: one GPU as rank 0 of a 4-rank pooled buffer (period
    4 N), the collective stood in for, the other ranks' chunks packed (once, from segment
    0) from this GPU's rows: every learn's draws equal the oracle's, segment 0's slots that
    rank 0 owns equal the literal loop's, and no chunk overflows."""
    checked, skipped = _run(0, 4, 6, 500, 30_011, 333, 3, gpu, sampler="philox", exchange="allgather", fused=True,
                            emulate=True)
    assert checked + skipped == 3 * SEG


def test_staged_replay_refuses_a_ring_older_than_one_segment(gpu, built_lib):
    from sacenv.replay import StagedReplay
    with pytest.raises(ValueError):
        StagedReplay(100, 128, 6, torch.zeros(11), mem_size=SEG * 100 + 1, seg=SEG, device=gpu)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, sampler="mt", exchange="allreduce", fused=False):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "sac-agent_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, _run(rank, world, 6, 1000, 30_011, 333, 3, torch.device("cuda", 0), sampler=sampler,
                          exchange=exchange, fused=fused)))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("sampler,exchange,fused", [("mt", "allreduce", False), ("philox", "allgather", False),
                                                    ("philox", "allgather", True)])
def test_staged_replay_two_ranks_equal_pooled_buffer(sampler, exchange, fused, gpu, built_lib):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q, sampler, exchange, fused)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert res[0] == (3 * SEG, 0) and res[1] is None, res


def test_bench_runner_exchange_equals_direct_staged_replay(gpu, built_lib):
    """bench's timed N>1 path (SegmentRunner with the SegmentExchange of --pooling
    sharded, at world 1) samples the same batches as the staged replay driven by
    hand (StagedReplay + segment_async(stage=...) + refill, one stream): the runner's
    segments must write the staged rows (a runner that stepped plain segments would
    gather stale rows)."""
    import bench
    from sacenv.replay import StagedReplay
    args = bench.parse(["--no-cpu-baseline", "--envs", "4096", "--replay-mem", "100003",
                        "--replay-batch", "257"])
    wl_a, wl_b = (bench.make_workload(args, 0, gpu) for _ in range(2))
    x = bench.make_exchange(args, wl_a, 0, 1, gpu)
    run = bench.SegmentRunner(args, wl_a, gpu, None, bench.SEG, x)
    env_b = wl_b.envs[0]
    rep = StagedReplay(env_b.num_envs, env_b.n_pad, args.experiment, env_b.first_obs_template(), rank=0,
                       world=1, mem_size=args.replay_mem, batch=args.replay_batch, seg=bench.SEG, seed=0,
                       device=gpu, sampler=args.sampler, exchange=args.exchange)
    assert (args.sampler, args.exchange) == ("philox", "allgather")   # bench's defaults
    rep.begin(env_b.obs)
    k = 0
    for g in range(3):
        k = run.segment(k, False)
        run.finish()
        sa = rep.stage_args(g)
        wl_b.segment_step(g * bench.SEG % bench.ACTION_STEPS, bench.SEG, stage=sa["stage"], marks=sa["marks"])
        wl_b.refill()
        rep.prepare(g + 1)
        want = rep.sample_segment(g)
        torch.cuda.synchronize()
        got = x.last
        assert len(got) == len(want) == bench.SEG
        for j in (0, 1, 77, bench.SEG - 1):
            for u, v in zip(got[j], want[j]):
                assert torch.equal(u, v), (g, j)
    rep.check()
    x.sampler.check()
