"""The driver's exact round-end bench command on the GPU (round 1 died on it).

Runs ``python bench.py --gpus 1 --steps 20 --warmup 5`` as a child process
(with a 1-second CPU-baseline budget) and checks the JSON line: rc 0, whole
segments executed, ``roofline`` and ``cpu_baseline`` present, and the timed
steps fit in the wall time of the run.
"""
import json
import os
import subprocess
import sys
import time

import pytest

from conftest import ROOT


@pytest.mark.gpu
def test_driver_bench_command():
    t0 = time.perf_counter()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "20",
                        "--warmup", "5", "--cpu-seconds", "1"],
                       capture_output=True, text=True, timeout=600, cwd=ROOT)
    wall = time.perf_counter() - t0
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    d = json.loads(line)
    # >= 8 timed segments, the warm-up past the clock boost, and the timed region lasts >= 1 s
    # (bench.MIN_TIMED_SECONDS, sized at the warm-up's post-boost rate)
    assert d["steps"] % 256 == 0 and d["steps"] >= 8 * 256 and d["n_gpus"] == 1
    assert d["warmup"] == 256 * 24
    assert d["ms_per_step"] * d["steps"] * 1e-3 >= 1.0
    assert d["value"] > 0 and d["unit"] == "env-steps/s"
    assert d["ms_per_step"] * d["steps"] * 1e-3 <= wall
    # every captured graph (4 action-table segments) ran once before the warm-up
    assert d["setup"]["graph_first_replays"] == 512
    rf = d["roofline"]
    # the persistent step is bound by FP64 instruction issue (PMC: profiles/*pmc_segment.json);
    # the byte figures stay beside it
    assert rf["bound"] == "fp64-issue" and rf["unit"] == "TFLOP/s" and 0 < rf["frac"] < 1
    assert 0 < rf["issue_floor_frac"] <= 1.05 and rf["kernel_avg_us"] > 0
    assert 0 < rf["hbm"]["frac"] < 1 and rf["hbm"]["unit"] == "GB/s"
    # the N>1 replay path at one GPU, measured on the same line, with the sampler it timed, and
    # the same with the collective's kernel stood in for
    rp, sd = d["replay_path"], d["replay_path_collective_standin"]
    assert rp["value"] > 0 and d["every_output"]["value"] > 0
    assert rp["sampler"] == "philox" and rp["exchange"] == "allgather"
    assert sd["value"] > 0 and sd["standin"]["workgroups"] == 16 and sd["standin"]["bytes"] > 20e6
    # one GPU as rank 0 of the 8-rank pooled buffer (the N = 8 line's per-rank work)
    rk = d["replay_path_rank_of_world"]
    assert rk["value"] > 0 and rk["world"] == 8 and 0 < rk["frac_of_value"] < 1.05
    assert 0 < rp["frac_of_value"] < 1.05
    if rf["kernel"].startswith("k_rollout"):  # the persistent launch: resident-state bytes headline
        assert abs(rf["bytes_per_env_step"] - (70 + 152 / 256)) < 1e-9
        assert rf["survey_222B"]["bytes_per_env_step"] == 222
    # the timed step includes its refill: never faster than the kernel alone
    assert rf["step_us_incl_refill"] >= rf["kernel_avg_us"]
    cb = d["cpu_baseline"]
    assert cb["value"] > 0 and cb["cores"] >= 1 and cb["kind"] == "port" and cb["one_core"] > 0
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        assert d["metric"] == json.load(f)["metric"]


def _two_rank_env():
    return dict(os.environ, SACENV_BENCH_BACKEND="gloo", SACENV_BENCH_ONE_DEVICE="1")


@pytest.mark.gpu
def test_bench_two_ranks_gloo_on_one_device():
    """The N>1 bench path (the staged replay exchange of the kernel-written transition rows,
    max-over-ranks timing; the all-gather beside it) as two processes sharing the one GPU
    over gloo, under the launcher the driver uses (torch.distributed.run). RCCL needs one
    device per rank; the driver's 8-GPU run is the RCCL one."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--gpus", "2", "--steps", "20", "--warmup", "5", "--envs", "8192"],
                       capture_output=True, text=True, timeout=600, cwd=ROOT, env=_two_rank_env())
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert d["n_gpus"] == 2 and d["steps"] % 256 == 0 and d["steps"] >= 8 * 256 and d["value"] > 0
    assert d["config"]["global_envs"] == 2 * 8192
    c = d["config"]["collective"]
    assert "gloo all_gather" in c and f"({d['steps'] // 256} in the timed region)" in c and "StagedReplay" in c
    po = d["pooling"]
    assert po["mode"] == "sharded" and po["exchanges_timed"] == d["steps"] // 256
    assert po["all_gather"]["value"] > 0 and po["no_exchange"]["value"] > 0


@pytest.mark.gpu
def test_bench_self_launch_two_ranks_on_one_device():
    """``python bench.py --gpus 2`` with no launcher: bench starts its own two ranks."""
    env = {k: v for k, v in _two_rank_env().items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "20",
                        "--warmup", "5", "--envs", "4096", "--exchange-segs", "1"],
                       capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["pooling"]["mode"] == "sharded" and d["value"] > 0


@pytest.mark.gpu
def test_bench_two_ranks_allreduce_exact_sampler():
    """The previous default, kept as options: the MT-exact draws and the SUM all-reduce."""
    env = {k: v for k, v in _two_rank_env().items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "20",
                        "--warmup", "5", "--envs", "4096", "--exchange-segs", "1", "--sampler", "mt",
                        "--exchange", "allreduce"],
                       capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert d["pooling"]["exchange"] == "allreduce" and "gloo SUM all_reduce" in d["config"]["collective"]
