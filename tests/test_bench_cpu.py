"""bench.py's control flow on the CPU with a stub stepper (no GPU).

The driver runs ``bench.py --gpus 1 --steps 20 --warmup 5`` at round end and
``--gpus N`` under torch.distributed.run on 8 GPUs; round 1's bench died on
the short command (no whole segment in the timed region). These tests drive
``run_bench`` -- the same timing loop, segment rounding, refill placement and
N>1 segment pooling -- with a stub workload at world sizes 1 and 2 (gloo).
"""
import json
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT

N_ENVS, N_PAD = 70, 128


class _StubEnv:
    """Stands in for VecBoatEnv: the record / terminal-obs regions the pool reads."""

    def __init__(self, rank):
        self.num_envs, self.n_pad = N_ENVS, N_PAD
        self.record = torch.zeros(50 * N_PAD, dtype=torch.uint8)
        self.final_obs_bytes = torch.zeros(44 * N_PAD, dtype=torch.uint8)
        self.rank, self.steps, self.refills, self.refill_at = rank, 0, 0, []

    def step_async(self, actions):
        assert actions.dtype == torch.float32 and actions.numel() == N_ENVS
        self.steps += 1
        self.record.fill_((self.steps + 31 * self.rank) % 251)
        self.final_obs_bytes.fill_((self.steps * 7 + self.rank) % 253)

    def refill(self):
        self.refills += 1
        self.refill_at.append(self.steps)


def _workload(bench, rank):
    from sacenv.dist import TransitionLayout
    env = _StubEnv(rank)
    actions = torch.rand((bench.ACTION_STEPS, N_ENVS), generator=torch.Generator().manual_seed(rank))
    lay = TransitionLayout(N_ENVS, N_PAD)

    def pooled_step(k, row):
        assert row.numel() == lay.nbytes
        env.step_async(actions[k % bench.ACTION_STEPS])
        row.fill_((env.steps * 3 + rank) % 255)

    return env, bench.Workload([env], env.step_async, env.refill, actions, pooled_step, lay.nbytes,
                               N_ENVS, bench.BYTES_PER_ENV_STEP * N_ENVS)


def _run(rank, world, argv):
    import bench
    args = bench.parse(argv)
    env, wl = _workload(bench, rank)
    out = bench.run_bench(args, rank, world, torch.device("cpu"), wl)
    return out, env


def test_driver_command_world1_rounds_to_whole_segments():
    out, env = _run(0, 1, ["--gpus", "1", "--steps", "20", "--warmup", "5"])
    assert out["steps"] == 8 * 256 and out["warmup"] == 512   # at least 8 timed, 2 warm-up segments
    assert out["requested"] == {"steps": 20, "warmup": 5, "rule": out["requested"]["rule"]}
    # every segment ends with its refill; timed region = eight whole segments (+ k_step segs after)
    assert all(s % 256 == 0 for s in env.refill_at), env.refill_at
    assert env.refill_at[:2] == [256, 512]
    assert out["value"] > 0 and out["ms_per_step"] > 0
    assert out["roofline"]["frac"] > 0 and out["roofline"]["kernel_avg_us"] > 0
    assert out["metric"].startswith("env-steps/sec (whole node), boat_env exp-6, 65 536 envs/GPU")
    json.dumps(out)


def test_metric_follows_the_config():
    import bench
    a = bench.parse(["--experiment", "1", "--envs", "4096"])
    assert "exp-1" in bench.metric_name(a) and "4 096 envs/GPU" in bench.metric_name(a)
    m = bench.parse(["--mixed"])
    assert "mixed batch" in bench.metric_name(m) and "32 768" in bench.metric_name(m)


@pytest.mark.parametrize("steps,warmup,n_timed", [(20, 5, 8), (300, 0, 8), (2100, 0, 9)])
def test_segment_rounding(steps, warmup, n_timed):
    out, env = _run(0, 1, ["--steps", str(steps), "--warmup", str(warmup), "--kernel-launches", "1"])
    assert out["steps"] == n_timed * 256
    # warmup segs + timed segs + 2 k_step-only segments (eager path), each with a refill
    assert env.refills == out["warmup"] // 256 + n_timed + 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dist_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "sac-agent_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out, env = _run(rank, world, ["--gpus", str(world), "--steps", "20", "--warmup", "5"])
        q.put((rank, out, env.steps, env.refills))
    finally:
        dist.destroy_process_group()


def test_driver_command_world2_gloo_segment_pooling():
    """The N>1 path (SegmentPool of full transitions) with the driver's short command."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dist_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=300) for _ in range(world)), key=lambda x: x[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    out = res[0][1]
    assert res[1][1] is None
    assert out["steps"] == 8 * 256 and out["n_gpus"] == 2
    assert out["value"] > 0
    assert "8 in the timed region" in out["config"]["collective"]
    assert "gloo" in out["config"]["collective"]
    # the row is the step kernel's 45-B/env transition row
    assert f"{45 * N_PAD} B per rank-step" in out["config"]["collective"]
    assert out["pooling"]["received_bytes_per_rank"] == (world - 1) * 45 * N_PAD * out["steps"]
    assert out["pooling"]["received_GBps_per_rank"] > 0
    # the no-exchange rate of the same segments, measured after the timed region
    ne = out["pooling"]["no_exchange"]
    sh = ne["sharded_exchange"]     # one all-reduce of a segment's 256 learn() batches
    assert sh["bytes_per_segment"] == 256 * 1024 * 26 * 4 and sh["allreduce_ms_per_segment"] > 0
    assert 0 < sh["value"] < ne["value"] * 1.01
    assert ne["value"] > 0 and ne["steps"] % 256 == 0 and ne["ms_per_step"] > 0
    for _, _, steps, refills in res:
        assert steps % 256 == 0 and refills == steps // 256
