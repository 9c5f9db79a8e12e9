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
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))
from bench_stub import N_PAD, workload as _stub_workload  # noqa: E402


def _workload(bench, rank):
    return _stub_workload(bench, rank)


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


def _dist_worker(rank, world, port, q, extra):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "sac-agent_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out, env = _run(rank, world, ["--gpus", str(world), "--steps", "20", "--warmup", "5", "--stub",
                                      "--replay-batch", "64", *extra])
        q.put((rank, out, env.steps, env.refills))
    finally:
        dist.destroy_process_group()


def _world2(extra):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dist_worker, args=(r, world, port, q, extra)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=300) for _ in range(world)), key=lambda x: x[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert res[1][1] is None
    for _, _, steps, refills in res:
        assert steps % 256 == 0 and refills == steps // 256
    return res[0][1]


def test_driver_command_world2_gloo_segment_gather():
    """The all-gather pooling (--pooling gather) with the driver's short command."""
    out = _world2(["--pooling", "gather"])
    assert out["steps"] == 8 * 256 and out["n_gpus"] == 2
    assert out["value"] > 0
    assert "8 in the timed region" in out["config"]["collective"]
    assert "gloo" in out["config"]["collective"]
    # the row is the step kernel's 53-B/env transition row
    assert f"{53 * N_PAD} B per rank-step" in out["config"]["collective"]
    po = out["pooling"]
    assert po["mode"] == "gather" and po["received_bytes_per_rank"] == 53 * N_PAD * out["steps"]
    assert po["received_GBps_per_rank"] > 0
    ne = po["no_exchange"]     # the no-exchange rate of the same segments, after the timed region
    assert ne["value"] > 0 and ne["steps"] % 256 == 0 and ne["ms_per_step"] > 0


def test_driver_command_world2_gloo_sharded_exchange():
    """The default N>1 pooling: each segment's rows staged per rank and the segment's
    learn() batches exchanged with one all-gather of each rank's packed rows, inside the
    timed region; the all-gather of every transition and no exchange measured beside it."""
    out = _world2([])
    assert out["steps"] == 8 * 256 and out["n_gpus"] == 2 and out["value"] > 0
    po = out["pooling"]
    assert po["mode"] == "sharded" and po["exchanges_timed"] == 8
    assert po["exchange"] == "allgather" and po["sampler"] == "philox"
    chunk = (-(-256 * 64 // 2) * 25 + 4) * 4
    assert po["bytes_per_segment"] == 2 * chunk and po["bus_bytes_per_rank"] == 8 * chunk
    assert "8 in the timed region" in out["config"]["collective"] and "all_gather" in out["config"]["collective"]
    assert "Philox" in out["config"]["collective"]
    assert po["xgmi"]["GBps_per_rank"] > 0
    ag = po["all_gather"]
    assert ag["value"] > 0 and ag["received_bytes_per_rank"] == 53 * N_PAD * ag["steps"]
    assert po["no_exchange"]["value"] > 0
    assert out["data"].startswith("stub")


def test_driver_command_world2_gloo_sharded_allreduce():
    """--exchange allreduce: the SUM all-reduce of the 1/N-dense batch words."""
    out = _world2(["--exchange", "allreduce", "--sampler", "mt"])
    po = out["pooling"]
    assert po["mode"] == "sharded" and po["exchange"] == "allreduce" and po["sampler"] == "mt"
    assert po["bytes_per_segment"] == 256 * 64 * 26 * 4
    assert po["bus_bytes_per_rank"] == 8 * 2 * (2 - 1) / 2 * 256 * 64 * 26 * 4
    assert "all_reduce" in out["config"]["collective"]


@pytest.mark.parametrize("argv,mode", [([], "sharded"), (["--launch", "step"], "gather"),
                                       (["--no-graph"], "gather"), (["--pooling", "none"], "none"),
                                       (["--mixed"], "gather")])
def test_sharded_pooling_needs_the_segment_launch(argv, mode):
    """the staged replay's rows are written by the persistent segment launch;
    --launch step / --no-graph at N>1 time the all-gather pooling instead (a KeyError in
    the timed loop before)."""
    import bench
    args = bench.parse(["--gpus", "2", *argv])
    _, wl = _workload(bench, 0)
    wl.segment_step = lambda *a, **k: None   # (a GPU workload has one)
    wl.segment_pools = not args.mixed
    assert bench.pooling_mode(args, 2, wl) == mode
    assert bench.pooling_mode(args, 1, wl) == "none"


def test_driver_command_world2_gloo_launch_step():
    """--gpus 2 --launch step: the runner steps k_step launches and the rows pooled
    (stub: the control flow of that combination end to end)."""
    out = _world2(["--launch", "step"])
    assert out["n_gpus"] == 2 and out["value"] > 0 and out["pooling"]["exchanges_timed"] == 8


def test_bench_self_launches_its_ranks():
    """python bench.py --gpus 2 with no launcher (WORLD_SIZE unset): bench starts its two
    rank processes itself; rank 0 prints the one JSON line."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--stub", "--steps", "20",
                        "--warmup", "5", "--replay-batch", "32", "--exchange-segs", "1"],
                       capture_output=True, text=True, env=env, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["pooling"]["mode"] == "sharded" and out["value"] > 0


def test_bench_self_launch_fails_loudly():
    """Ranks that die end the run with a non-zero status and no line."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--stub",
                        "--pooling", "gather", "--pool-every", "7"], capture_output=True, text=True, env=env,
                       timeout=300, cwd=ROOT)
    assert r.returncode != 0 and "must divide" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
