"""Benchmark: env-steps/s of the HIP boat env (BASELINE.json metric).

Workload (BASELINE.json configs[2] at N=1, configs[3] at N>1): boat_env
experiment 6 (random wind in all directions), 65 536 envs per GPU,
test_mode 0 (actions drive the rudder), actions U(-1,1) f32 pre-generated as
a [512, N] table in HBM, episodes truncated at 500 steps and auto-reset in
the step kernel (early terminations too). One "step" = one BoatEnv.step over
all envs of the rank (+ at N>1 pooling the step's full transitions -- record,
action and terminal obs -- for a shared replay buffer over RCCL).

    python bench.py [--gpus N] [--steps K] [--warmup W]

Timing. Steps run in whole 256-step segments: each segment is one hipGraph of
256 step launches followed by the slot refill (k_need_masks + k_refill +
k_refill_fit: the RNG draws and spline fits of the episodes that replace the
ended ones), which the engine needs at least every 256 steps. W and K are
rounded UP to whole segments (at least one each), so the timed region always
starts on a segment boundary and always holds its share of refills; the JSON
``steps`` / ``warmup`` are the step counts actually executed (the requested
ones are in ``requested``). The timed region is bracketed by barrier +
synchronize; value = all envs x steps / max-over-ranks time.

Roofline: algorithmic bytes per env-step x envs, over the kernel's average
per-step duration from HIP events on the kernel's stream (refills excluded;
they are in ``ms_per_step``). ``--launch step``: SURVEY.md §8(d)'s 222 B per
boat env-step (state read and written every step). ``--launch segment`` (the
default): the same components with the state resident in registers for the
256-step launch, 70 B per step + 152 B per launch (SURVEY's 222-B equivalent
rate is reported beside it). ``traffic`` = HBM bytes per step from the
committed rocprofv3 PMC passes (tools/pmc.sh).

cpu_baseline: SURVEY.md §8(d) C1 -- the reference step restated
(oracle/boat_oracle.py) at ONE env per process, as the reference runs, on one
core and on all cores of the lease (tools/cpu_c1.py, a child process), for
the bench's experiment; the vectorised numpy port on the bench's env count is
a secondary field.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import subprocess
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "sac-agent_amd"))

BYTES_PER_ENV_STEP = 222      # state r+w 152, action 4, wind 16, obs 44, reward 4, done+term 2
SEG_MIN_BYTES = 70 + 152 / 256  # the same with the state in registers for a 256-step persistent launch
TOY_BYTES = {"parachute": 86, "car": 102}
# the toys in the persistent mixed launch: obs 8 + reward 4 + done/term 2 per step, state r+w once
TOY_SEG_BYTES = {"parachute": 14 + 72 / 256, "car": 14 + 88 / 256}
HBM_PEAK = 8.0e12             # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
EPISODE_STEPS = 500
SEG = 256              # step launches per refill (sacenv _lib.REFILL_PERIOD); one graph per segment
ACTION_STEPS = 512     # the pre-generated action table cycles every 512 steps (2 segments)
TRANS_ROW = "53-B/env transition row (s' f32 x 11, reward, action, term; done = term != 0)"


def metric_name(args) -> str:
    """BASELINE.json's metric for the default workload; the same wording for the others."""
    def num(n: int) -> str:
        return f"{n:,}".replace(",", " ")
    if args.mixed:
        return (f"env-steps/sec (whole node), mixed batch boat_env exp-{args.experiment} + "
                f"toy_parachute + toy_car, {num(args.mixed_envs)} envs each/GPU")
    return (f"env-steps/sec (whole node), boat_env exp-{args.experiment}, "
            f"{num(args.envs)} envs/GPU at 1/2/4/8 MI355X")


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2048)
    ap.add_argument("--warmup", type=int, default=512)
    ap.add_argument("--envs", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--min-seconds", type=float, default=MIN_TIMED_SECONDS,
                    help="the timed region lasts at least this long (whole segments; GPU runs only)")
    ap.add_argument("--experiment", type=int, default=6)
    ap.add_argument("--no-graph", action="store_true", help="eager per-step launches (--launch step)")
    ap.add_argument("--launch", choices=("segment", "step"), default="segment",
                    help="segment: one persistent sacenv_boat_segment launch per 256 steps (state in "
                         "registers, actions behind per-wave flags); step: one k_step launch per step, "
                         "256 of them per hipGraph replay")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="total CPU-baseline budget (4 C1 legs + the vectorised port)")
    ap.add_argument("--kernel-launches", type=int, default=256)
    ap.add_argument("--test-mode", type=int, default=0, help="1 = rudder frozen (no terminations)")
    ap.add_argument("--helpers", type=int, default=None,
                    help="workgroups of a refill draw launch (default: VecBoatEnv's, 3/16 of the envs)")
    ap.add_argument("--mixed", action="store_true",
                    help="BASELINE configs[4]: boat exp-6 + toy_parachute + toy_car in one launch")
    ap.add_argument("--mixed-envs", type=int, default=32768, help="envs per type per GPU (--mixed)")
    ap.add_argument("--no-autoreset", action="store_true",
                    help="diagnostic: no in-kernel auto-reset (ended envs keep stepping)")
    ap.add_argument("--rollout", type=int, default=0,
                    help="K > 0: open-loop K-step rollouts (sacenv_boat_rollout), a separate line")
    ap.add_argument("--pooling", choices=("sharded", "gather", "none"), default="sharded",
                    help="N>1: sharded = the pooled replay buffer sampled out of each rank's staged "
                         "segments, one SUM all-reduce of the segment's learn() batches (StagedReplay; the "
                         "all-gather rate is measured beside it); gather = all-gather every transition per "
                         "256-step segment (configs[3]'s literal exchange); none = no exchange")
    ap.add_argument("--sampler", choices=("philox", "mt"), default="philox",
                    help="the staged replay's index draws: philox = counter-based (np.random.choice's "
                         "distribution per learn, every draw independent: one parallel launch per segment); "
                         "mt = the reference stream's exact draws (one MT19937 chain per segment)")
    ap.add_argument("--exchange", choices=("allgather", "allreduce"), default="allgather",
                    help="N>1 --pooling sharded: allgather = each rank's own sampled rows packed with their "
                         "slots, one all_gather of the chunks; allreduce = one SUM all-reduce of the "
                         "1/N-dense batches (twice the bytes per rank)")
    ap.add_argument("--channels", type=int, default=16,
                    help="RCCL channel cap for N>1 (NCCL_MAX_NCHANNELS unless set): the collective's "
                         "workgroups sharing CUs with the segment launch; also the stand-in's workgroups")
    ap.add_argument("--standin-gbps", type=float, default=250.0,
                    help="N=1 collective stand-in: the per-rank rate its transfer is modelled at (it stays "
                         "resident for bytes / rate)")
    ap.add_argument("--standin-world", type=int, default=8,
                    help="N=1 collective stand-in: the world size whose per-rank traffic it moves")
    ap.add_argument("--replay-mem", type=int, default=1_000_000,
                    help="pooled ReplayBuffer(max_size) (configs/original_config.yaml: 1 000 000)")
    ap.add_argument("--replay-batch", type=int, default=1024, help="learn() batch (agent.batch_size: 1024)")
    ap.add_argument("--exchange-segs", type=int, default=4,
                    help="segments per side measurement after the timed region (the other exchanges)")
    ap.add_argument("--stub", action="store_true",
                    help="CPU control-flow rehearsal: a stub workload, no kernels (tools/bench_stub.py); "
                         "the line says data: stub")
    ap.add_argument("--pool-every", type=int, default=SEG,
                    help="N>1 gather pooling: steps per all-gather (1 = one all-gather per step, "
                         "SURVEY.md §8(e); 256 = one per segment, overlapped with the next)")
    ap.add_argument("--event-every", type=int, default=4,
                    help="time every E-th timed segment's launch (the first always) with HIP events "
                         "for roofline.kernel_avg_us: each pair puts a stream marker on both sides of "
                         "the launch (measured: every segment 1.78 us/step, every 4th 1.74)")
    ap.add_argument("--no-every-output", action="store_true",
                    help="skip the every-output rollout measurement after the timed region (PMC passes: its "
                         "k_rollout launches would mix into the segment kernel's counters)")
    ap.add_argument("--closed-loop", action="store_true",
                    help="a separate line: the SAC actor choosing every step's actions on the device, handing "
                         "off to the persistent env launch through per-wave flags (sacenv.closed_loop)")
    ap.add_argument("--train", action="store_true",
                    help="a separate line: main.py:78-90's whole loop per step on the device -- NativeSAC "
                         "choose_action, the env step, the transitions stored, one learn() on a sampled batch")
    ap.add_argument("--episode-steps", type=int, default=EPISODE_STEPS,
                    help="truncation length (0 = none)")
    return ap.parse_args(argv)


MIN_TIMED_SEGS = 8   # the timed region holds at least 2 048 steps
MIN_TIMED_SECONDS = 1.0  # and lasts at least ~1 s (whole segments, sized from the warm-up's rate), so
                         # an outside sampler of GPU activity sees the timed phase
                         # (--min-seconds)
TIMED_MARGIN = 1.15  # segments for 1.15 x --min-seconds at the warm-up's post-boost rate: the timed region
                     # lasts >= --min-seconds (round 5 sized it from the whole warm-up, pre-boost, and
                     # timed 0.83 s)
WARM_BOOST_SEGS = 24  # GPU warm-up: the clock boosts after ~20 launches
MIN_WARMUP_SEGS = 2  # and at least 512 warm-up steps: the driver's --steps 20 --warmup 5 then
                     # times the default line's region (the episode-length transient of the
                     # first ~1 000 steps -- every env starts at step 0 -- is behind it)


def segs(n_steps: int) -> int:
    """Whole segments covering n_steps (at least one)."""
    return max(1, -(-int(n_steps) // SEG))


def warm_segs(n_steps: int) -> int:
    """Warm-up segments for --warmup n: whole segments, at least MIN_WARMUP_SEGS."""
    return max(MIN_WARMUP_SEGS, segs(n_steps))


def timed_segs(n_steps: int) -> int:
    """Timed segments for --steps n: whole segments, at least MIN_TIMED_SEGS. A single
    128-step segment (round 3) was a ~0.25-ms region in which the first launch's submission
    after an idle stream and the closing synchronize (~44 us) were 13 % of the time."""
    return max(MIN_TIMED_SEGS, segs(n_steps))


# ---------------------------------------------------------------- distributed
def init_dist(n_gpus: int, stub: bool = False, channels: int = 16):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != n_gpus:
        raise SystemExit(f"--gpus {n_gpus} but WORLD_SIZE={world}")
    if stub:
        dev = torch.device("cpu")
    else:
        if os.environ.get("SACENV_BENCH_ONE_DEVICE"):  # rehearsal of the N>1 path on a 1-GPU box
            local = 0
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = "gloo" if stub else os.environ.get("SACENV_BENCH_BACKEND", "nccl")  # gloo: rehearsal
        if backend == "nccl":
            # the collective's workgroups share CUs with the persistent segment launch's owner
            # waves (one per SIMD): cap its channels (read by RCCL at communicator creation)
            os.environ.setdefault("NCCL_MAX_NCHANNELS", str(int(channels)))
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    return rank, world, dev


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n: int, argv) -> int:
    """``--gpus N`` with no launcher (WORLD_SIZE unset): start N rank processes of this
    script (RANK = LOCAL_RANK = r, WORLD_SIZE = N, a free 127.0.0.1 port) and wait for
    them. The parent touches no GPU (nothing here initialises HIP), rank 0 prints the
    line on the inherited stdout, and the exit status is the first failing rank's. A
    rank that fails ends the others (their own PIDs), so a broken collective cannot
    leave the rest waiting on it."""
    env = dict(os.environ, WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    procs = []
    for r in range(n):
        e = dict(env, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=e))
    rc = 0
    live = list(procs)
    while live:
        time.sleep(0.2)
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:      # the others would wait on the failed rank's collectives
                    q.terminate()
    for p in procs:
        try:
            p.wait(timeout=30)
        except subprocess.TimeoutExpired:
            p.kill()
    return rc if rc > 0 else (1 if rc else 0)


XGMI_LINK_GBPS = 153.0  # the task brief's MI355X xGMI figure: 7 links x ~153 GB/s per GPU


def dist_info(world: int, dev) -> dict | None:
    """N>1: what ran the collectives (backend, RCCL version, each rank's device)."""
    if world <= 1:
        return None
    import torch.distributed as dist
    me = {"rank": dist.get_rank(), "local_rank": int(os.environ.get("LOCAL_RANK", "0")),
          "device": str(dev)}
    if dev.type == "cuda":
        pr = torch.cuda.get_device_properties(dev)
        me["device_name"] = pr.name
        me["pci_bus_id"] = getattr(pr, "pci_bus_id", None)
    ranks = [None] * world
    dist.all_gather_object(ranks, me)
    backend = dist.get_backend()
    ver = None
    if backend == "nccl":
        try:
            v = torch.cuda.nccl.version()
            ver = ".".join(map(str, v)) if isinstance(v, tuple) else str(v)
        except Exception as exc:  # noqa: BLE001
            ver = f"unavailable: {exc}"
    return {"world_size": world, "backend": "RCCL (nccl)" if backend == "nccl" else backend,
            "rccl_version": ver, "rccl_max_channels": os.environ.get("NCCL_MAX_NCHANNELS") if backend == "nccl"
            else None, "ranks": ranks}


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


class _Clock:
    """A HIP event on the stepping stream (GPU) or a host clock (CPU stub runs)."""

    def __init__(self, dev):
        self.cuda = dev.type == "cuda"
        self.ev = torch.cuda.Event(enable_timing=True) if self.cuda else None
        self.t = None

    def record(self, stream=None):
        if self.cuda:
            self.ev.record(stream)
        else:
            self.t = time.perf_counter()

    def ms_to(self, other: "_Clock") -> float:
        return self.ev.elapsed_time(other.ev) if self.cuda else (other.t - self.t) * 1e3


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


# ---------------------------------------------------------------- cpu baseline
def cpu_baseline(args, n_envs: int) -> dict:
    """SURVEY.md §8(d) C1 on this host: tools/cpu_c1.py (a child process; the
    oracle at one env per process, 1 core and all cores of the lease, exp 1 and
    the bench's experiment), plus the vectorised port on the bench's shape."""
    budget = max(2.0, float(args.cpu_seconds))
    exps = sorted({1, int(args.experiment)})
    per_leg = budget * 0.8 / (3 * len(exps))
    cmd = [sys.executable, os.path.join(ROOT, "tools", "cpu_c1.py"), "--seconds", f"{per_leg:.2f}",
           "--experiments", ",".join(map(str, exps)), "--max-procs", "16", "--mode", "scalar",
           "--numpy-one-core"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        raise RuntimeError(f"cpu_c1 failed: {r.stderr[-2000:]}")
    c1 = json.loads(r.stdout.strip().splitlines()[-1])
    leg = c1["experiments"][str(args.experiment)]
    out = {"value": leg["all_cores"]["env_steps_per_s"], "unit": "env-steps/s",
           "cores": leg["all_cores"]["procs"], "kind": "port",
           "sample": (f"SURVEY.md §8(d) C1 in §7.2's scalar N=1 mode: oracle/boat_scalar.py (BoatEnv.step, "
                      f"boat_env.py:67-115, restated with Python floats + math, f64; per-episode wind "
                      f"tables materialised at reset as the reference does), exp {args.experiment}, ONE "
                      f"env per process (as the reference runs), {leg['all_cores']['procs']} processes "
                      f"pinned one per core, U(-1,1) actions, reset on done or at 500 steps, "
                      f"{per_leg:.1f} s per leg"),
           "one_core": leg["one_core"]["env_steps_per_s"],
           "one_core_numpy_n1": leg.get("one_core_numpy_n1", {}).get("env_steps_per_s"),
           "c1": c1}
    if not args.mixed:
        out["vectorised_port"] = _vectorised_port(n_envs, budget * 0.2, args.experiment)
    return out


def _vectorised_port(n_envs: int, seconds: float, experiment: int) -> dict:
    """The numpy oracle vectorised over the bench's env count, 1 thread (secondary)."""
    import numpy as np
    try:
        from threadpoolctl import threadpool_limits
        ctx = threadpool_limits(limits=1)
    except Exception:  # noqa: BLE001
        import contextlib
        ctx = contextlib.nullcontext()
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from boat_oracle import OracleConfig, OracleVecBoat
    n = min(n_envs, 16384)
    with ctx:
        ora = OracleVecBoat(OracleConfig(experiment=experiment, test_mode=0),
                            np.arange(n, dtype=np.uint64), max_episode_steps=EPISODE_STEPS)
        acts = np.random.default_rng(0).uniform(-1, 1, (64, n)).astype(np.float32)
        ora.step(acts[0])
        steps, t0 = 0, time.perf_counter()
        while True:
            ora.step(acts[steps % 64])
            steps += 1
            el = time.perf_counter() - t0
            if el >= seconds and steps >= 3:
                break
    return {"value": n * steps / el, "unit": "env-steps/s", "cores": 1,
            "sample": f"oracle/boat_oracle.py vectorised over {n} envs x {steps} steps ({el:.1f} s), 1 thread"}


def load_traffic(n_envs: int, experiment: int, launch: str = "step"):
    """Per-step HBM bytes of the timed kernel from the committed rocprofv3 PMC summary
    (tools/pmc.sh -> profiles/<round>_pmc_k_step.json or _pmc_segment.json, newest
    round first) for this workload shape, or None."""
    import glob
    pat = "*pmc_segment.json" if launch == "segment" else "*pmc_k_step.json"
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", pat)), reverse=True):
        try:
            d = json.load(open(path))
        except Exception:  # noqa: BLE001
            continue
        key = "hbm_bytes_per_step" if launch == "segment" else "hbm_bytes_per_launch"
        if int(d.get("envs", -1)) == n_envs and int(d.get("experiment", 6)) == experiment and key in d:
            # per step of all envs (a k_step launch; 1/SEG of a persistent launch)
            return {"hbm_bytes_per_launch": float(d[key]), "source": os.path.relpath(path, ROOT)}
    return None


FP64_VECTOR_PEAK = 78.6e12   # MI355X datasheet FP64 vector: 256 CUs x 4 SIMDs x 16 FMA lanes x 2 x 2.4 GHz
# measured ceilings (tools/ubench/f64_latency.hip, profiles/r04_ubench_*.txt): v_fma_f64 issue at one
# wave per SIMD 5.1 shader cycles per wave instruction (dependent 5.8), at two waves 3.5 per SIMD;
# 64-bit moves, conversions, rndne/ldexp/fract and AGPR reads ~8, v_readfirstlane ~24 (valu_mix.hip)


def load_compute(n_envs: int, experiment: int, kernel_s: float):
    """The step's FP64 VALU roofline from the committed PMC passes (tools/pmc.sh ->
    profiles/<round>_pmc_segment.json, newest first): VALU instructions and FP64
    flops per wave-step, the achieved FP64 rate at this run's kernel time against
    the datasheet peak, and the single-wave issue floor of that instruction count."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_segment.json")), reverse=True):
        try:
            d = json.load(open(path))
        except Exception:  # noqa: BLE001
            continue
        if int(d.get("envs", -1)) != n_envs or int(d.get("experiment", 6)) != experiment:
            continue
        pw, K = d["per_wave"], float(d["steps_per_launch"])
        valu = pw["INSTS_VALU"] / K
        salu = pw["INSTS_SALU"] / K
        flops = (2 * pw["INSTS_VALU_FMA_F64"] + pw["INSTS_VALU_MUL_F64"] + pw["INSTS_VALU_ADD_F64"]) / K
        achieved = flops * n_envs / kernel_s
        out = {"unit": "TFLOP/s (FP64 vector)", "achieved": achieved / 1e12, "peak": FP64_VECTOR_PEAK / 1e12,
               "frac": achieved / FP64_VECTOR_PEAK,
               "fp64_flops_per_env_step": flops, "valu_per_wave_step": valu, "salu_per_wave_step": salu,
               "f64_valu_per_wave_step": (pw["INSTS_VALU_FMA_F64"] + pw["INSTS_VALU_MUL_F64"]
                                          + pw["INSTS_VALU_ADD_F64"]) / K,
               "source": os.path.relpath(path, ROOT)}
        life, issue = pw.get("WAVE_CYCLES"), pw.get("ACTIVE_INST_ANY")
        if life and issue and d.get("trace_avg_ns_per_step"):
            # SQ cycle counters tick once per 4 shader cycles; the clock they imply over
            # the profiled launches' per-step time (a lower bound: a wave lives a little
            # less than its launch)
            clk = 4.0 * life / K / (d["trace_avg_ns_per_step"] * 1e-9)
            floor = 4.0 * issue / K / clk
            out.update({
                "issue_frac_of_wave_life": issue / life, "wait_frac_of_wave_life": pw.get("WAIT_ANY", 0.0) / life,
                "ifetch_frac_of_wave_life": pw.get("WAIT_INST_ANY", 0.0) / life,
                "clock_ghz_implied": clk / 1e9,
                "issue_floor_us_per_step": floor * 1e6, "issue_floor_frac": floor / kernel_s,
                "note": "one owner wave per SIMD issues in order, one instruction per 4-cycle issue slot at "
                        "best (f64 VALU ~5 cycles), so the step is bound by its instruction stream, not by HBM "
                        "bytes (counter traffic is ~0.1 of the byte figure) nor by FP64 throughput; "
                        "issue_floor = the measured issue cycles (SQ_ACTIVE_INST_ANY x 4) per step at the "
                        "implied clock; the rest of a wave's life is dependency waits (wait_frac) and "
                        "instruction fetch"})
        return out
    return None


# ---------------------------------------------------------------- workload
class Workload:
    """What the timing loop drives: ``stepper(actions_row)`` enqueues one step of
    every env of the rank, ``pooled_step(k, row)`` step k writing its pooled
    transition row (N>1; ``row_bytes`` per step), ``refill()`` the slot refill,
    ``envs`` the env objects."""

    def __init__(self, envs, stepper, refill, actions, pooled_step, row_bytes, per_gpu_envs,
                 bytes_per_launch, segment_step=None):
        self.envs, self.stepper, self.refill, self.actions = envs, stepper, refill, actions
        self.pooled_step, self._row_bytes = pooled_step, int(row_bytes)
        self.per_gpu_envs, self.bytes_per_launch = per_gpu_envs, bytes_per_launch
        # segment_step(k0, n, trans=None): steps k0 .. k0+n-1 in one persistent launch
        self.segment_step = segment_step
        self.segment_pools = True   # segment_step can write pooled transition rows

    def row_bytes(self) -> int:
        return self._row_bytes


def make_workload(args, rank: int, dev) -> Workload:
    from sacenv import VecBoatEnv, _lib
    from sacenv.dist import TransitionLayout
    assert SEG == _lib.REFILL_PERIOD
    N = args.mixed_envs if args.mixed else args.envs
    env = VecBoatEnv({"base_settings": {"experiment": args.experiment, "test_mode": args.test_mode}},
                     N, seed=0, device=dev, autoreset=not args.no_autoreset,
                     max_episode_steps=args.episode_steps,
                     env_id_offset=rank * N, n_helpers=args.helpers, auto_refill=False)
    env.reset()
    refill = env.refill if not args.no_autoreset else (lambda: None)
    envs, stepper = [env], env.step_async
    toys = []
    if args.mixed:
        from sacenv.toys import CarEnv, MixedBatch, ParachuteEnv
        toys = [ParachuteEnv(num_envs=N, device=dev, max_episode_steps=args.episode_steps),
                CarEnv(num_envs=N, device=dev, max_episode_steps=args.episode_steps)]
        envs += toys
        mixed = MixedBatch(env, toys)
        stepper = mixed.step_async
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    actions = torch.rand((ACTION_STEPS, N), generator=g, device=dev, dtype=torch.float32) * 2 - 1
    lay = TransitionLayout(N, env.n_pad, args.experiment)
    toy_bytes = [t.record.numel() + t.final_obs_bytes.numel() for t in toys]
    row_bytes = lay.nbytes + sum(toy_bytes)

    def pooled_step(k: int, row: torch.Tensor):
        # the boat's transition row, written by the step launch itself into the
        # pooling buffer (sacenv_boat_step_pooled / sacenv_mixed_step_pooled);
        # the toys' records and terminal obs copied behind it (open-loop toys
        # take no action, and a fresh toy's first obs is fixed)
        a = actions[k % ACTION_STEPS]
        if toys:
            mixed.step_async(a, row[: lay.nbytes])
            o = lay.nbytes
            for t in toys:
                for part in (t.record, t.final_obs_bytes):
                    row[o: o + part.numel()].copy_(part)
                    o += part.numel()
        else:
            env.step_pooled_async(a, row[: lay.nbytes])

    # the persistent launch's action hand-off: every row of the table is published
    # (the open-loop case of sacenv_boat_segment's per-wave flags; each wave still
    # reads its flag every step)
    ready = torch.full((env.n_pad // 64,), 0x7FFFFFFF, dtype=torch.int32, device=dev)

    import ctypes as C
    seg_fn, a0, astride = env.lib.sacenv_boat_segment, actions.data_ptr(), actions.stride(0)
    # the arguments are built right here (table [512, N] f32 contiguous, one flag per owner wave)
    assert actions.is_contiguous() and ready.numel() == env.n_pad // 64

    def segment_step(k0: int, n: int, trans=None, stage=None, marks=None):
        # sacenv_boat_segment (VecBoatEnv.segment_async without its per-call Python
        # checks): the timed loop pays one ctypes call
        r0 = k0 % ACTION_STEPS
        assert r0 + n <= ACTION_STEPS
        if trans is not None and trans.numel() < (n - 1) * row_bytes + lay.nbytes:
            raise ValueError("pooled rows buffer too small")
        if stage is not None and (stage.numel() < n * 64 * env.n_pad or (marks is not None and marks.numel() < env.n_pad * -(-n // 64))):
            raise ValueError("staged rows / marks buffer too small")
        _lib.check(seg_fn(env._pp, env._ptr, C.c_void_p(a0 + 4 * r0 * astride), astride, n, ready.data_ptr(),
                          None, 0, None if trans is None else trans.data_ptr(),
                          0 if trans is None else row_bytes, None if stage is None else stage.data_ptr(),
                          None if marks is None else marks.data_ptr(), torch.cuda.current_stream(dev).cuda_stream))

    if args.mixed:
        # the whole batch as ONE persistent launch per segment (sacenv_mixed_segment: the boat's
        # open loop + each toy wave's loop, state in registers); pooled rows go through the
        # per-step launches (graph mode) instead
        mix_fn, tp, ta = env.lib.sacenv_mixed_segment, mixed._tp, mixed._ta

        def segment_step(k0: int, n: int, trans=None):  # noqa: F811
            if trans is not None:
                raise ValueError("the persistent mixed launch writes no pooled rows")
            r0 = k0 % ACTION_STEPS
            assert r0 + n <= ACTION_STEPS
            _lib.check(mix_fn(env._pp, env._ptr, C.c_void_p(a0 + 4 * r0 * astride), astride, n, tp, ta, len(toys),
                              torch.cuda.current_stream(dev).cuda_stream))

    bytes_launch = BYTES_PER_ENV_STEP * N + (sum(TOY_BYTES.values()) * N if args.mixed else 0)
    wl = Workload(envs, stepper, refill, actions, pooled_step, row_bytes, N * len(envs), bytes_launch,
                  segment_step)
    wl.segment_pools = not args.mixed
    return wl


# ---------------------------------------------------------------- segments
class SegmentRunner:
    """Runs whole segments of the workload: steps k0 .. k0+SEG-1 (actions row k %
    ACTION_STEPS), then the slot refill, then (N>1) the pooling of the segment's
    transition rows. With a GPU and no ``--no-graph`` the SEG step launches of a
    segment are ONE hipGraph replay (one graph per segment of the action table and
    staging buffer); else eager launches. ``prepare()`` warms up and replays every
    captured graph once (its device upload), and runs the same steps eagerly in
    eager mode, so a graph runner and an eager runner of the same workload execute
    the same step sequence (tests/test_bench_path_gpu.py holds them bit-identical).

    ``pool_every`` P (N>1): the rows of P consecutive steps go out in one
    all-gather: P = SEG stages a segment's rows inside its graph and gathers them
    after it (``SegmentPool``, on a side stream); P < SEG (e.g. 1, SURVEY.md §8(e)'s
    one all-gather per step) steps eagerly and gathers every P steps."""

    def __init__(self, args, wl: Workload, dev, pool=None, pool_every: int = SEG, exchange=None):
        if SEG % pool_every:
            raise ValueError(f"--pool-every must divide {SEG}")
        self.args, self.wl, self.dev, self.pool = args, wl, dev, pool
        self.exchange = exchange   # sacenv.dist.SegmentExchange (the staged replay's exchange)
        self.pool_every = int(pool_every)
        # launch mode: "segment" (one persistent launch per segment, or per P steps
        # when pooling every P), "graph" (SEG k_step launches per hipGraph replay),
        # "eager" (SEG k_step launches)
        # (the mixed batch: sacenv_mixed_segment; with pooled rows it steps per launch)
        rows = pool is not None or exchange is not None
        want_seg = (getattr(args, "launch", "step") == "segment" and not args.no_graph
                    and wl.segment_step is not None and (not rows or wl.segment_pools))
        self.mode = ("segment" if want_seg and dev.type == "cuda" else
                     "graph" if (dev.type == "cuda" and not args.no_graph and exchange is None
                                 and (pool is None or pool_every == SEG))
                     else "eager")
        self.use_graph = self.mode == "graph"
        self.st = torch.cuda.current_stream(dev) if dev.type == "cuda" else None
        self.graphs = None
        self.first_replays = 0
        self.seg_events: list = []
        self._clocks: list = []   # pre-created events for the timed segments (no creation inside)
        self.event_every = max(1, int(getattr(args, "event_every", 1)))
        self.timed_segments = 0

    def reserve_clocks(self, n: int) -> None:
        """Create the timing events of n timed launches ahead of the timed region."""
        self._clocks = [(_Clock(self.dev), _Clock(self.dev)) for _ in range(n)]

    def _clock_pair(self):
        return self._clocks.pop() if self._clocks else (_Clock(self.dev), _Clock(self.dev))

    def _steps(self, k0: int, with_pool: bool, buf=None, on_step=None, timed: bool = False) -> None:
        """The SEG steps of one segment, enqueued (captured, eager or persistent)."""
        wl, p = self.wl, self.pool if with_pool else None
        x = self.exchange if with_pool else None
        if x is not None:   # the segment writes the staged replay's rows
            sa = x.stage_args()
            if self.mode == "segment":
                wl.segment_step(k0, SEG, stage=sa["stage"], marks=sa["marks"])
                return
            rows, rb = sa["rows"], wl.row_bytes()   # (the CPU stub: pooled rows per step)
            for j, k in enumerate(range(k0, k0 + SEG)):
                wl.pooled_step(k, rows[j * rb:(j + 1) * rb])
                if on_step is not None:
                    on_step(k)
            return
        if self.mode == "segment":
            if p is None:
                wl.segment_step(k0, SEG)
                return
            P = self.pool_every
            for j0 in range(0, SEG, P):  # one launch per all-gather group
                if P < SEG:
                    p.begin()
                wl.segment_step(k0 + j0, P, trans=p.stage[p.buf if buf is None else buf][: P * p.rb])
                if P < SEG:
                    p.fill = P
                    p.flush()
            return
        for j, k in enumerate(range(k0, k0 + SEG)):
            if p is None:
                wl.stepper(wl.actions[k % ACTION_STEPS])
            elif self.pool_every == SEG:
                wl.pooled_step(k, p.row(j, buf))
            else:  # P < SEG: eager, one all-gather per P steps
                jj = j % self.pool_every
                if jj == 0:
                    p.begin()
                wl.pooled_step(k, p.row(jj))
                if jj == self.pool_every - 1:
                    p.fill = self.pool_every
                    p.flush()
            if on_step is not None:
                on_step(k)

    def _capture(self, k0: int, buf: int, with_pool: bool):
        gr = torch.cuda.CUDAGraph()
        # thread_local: a collective library thread querying its events while this
        # thread captures must not invalidate the capture
        with torch.cuda.graph(gr, capture_error_mode="thread_local"):
            self._steps(k0, with_pool, buf)
        return gr

    def capture_all(self, with_pool: bool) -> None:
        bufs = (0, 1) if with_pool and self.pool is not None else (0,)
        self.graphs = [[self._capture(base, b, with_pool and self.pool is not None) for b in bufs]
                       for base in range(0, ACTION_STEPS, SEG)]

    def prepare(self, on_step=None) -> None:
        """Warm the launch path (3 steps + a refill), capture, and run every captured
        graph once (each followed by its refill) before the warm-up: a graph's first
        replay carries its upload to the device, which the driver's short --steps 20
        --warmup 5 would otherwise put into the timed region. Eager mode runs the
        same steps."""
        wl, dev = self.wl, self.dev
        if dev.type != "cuda":
            return
        if self.mode == "segment":  # the same steps as the graph and eager modes
            wl.segment_step(0, 3)
            wl.refill()
            for base in range(0, ACTION_STEPS, SEG):
                wl.segment_step(base, SEG)
                wl.refill()
                self.first_replays += SEG
            _sync(dev)
            return
        if self.use_graph:
            s = torch.cuda.Stream(device=dev)
            s.wait_stream(self.st)
            with torch.cuda.stream(s):
                for k in range(3):
                    wl.stepper(wl.actions[k])
            self.st.wait_stream(s)
        else:
            for k in range(3):
                wl.stepper(wl.actions[k])
                if on_step is not None:
                    on_step(k)
        wl.refill()
        _sync(dev)
        if self.use_graph:
            self.capture_all(with_pool=self.pool is not None)
            for gset in self.graphs:
                for gr in gset:
                    gr.replay()
                    wl.refill()
                    self.first_replays += SEG
        else:
            nbuf = 2 if self.pool is not None and self.pool_every == SEG else 1
            for base in range(0, ACTION_STEPS, SEG):
                for b in range(nbuf):
                    self._steps(base, False, on_step=on_step)  # the graph replays' steps
                    wl.refill()
                    self.first_replays += SEG
        _sync(dev)

    def finish(self) -> None:
        """The stepping stream waits for everything a segment left in flight (the last
        all-gathers / replay exchanges)."""
        if self.pool is not None:
            self.pool.wait()
        if self.exchange is not None:
            self.exchange.wait()

    def segment(self, k0: int, timed: bool = False, with_pool: bool = True, on_step=None) -> int:
        """Steps k0 .. k0+SEG-1 (k0 % SEG == 0), then the refill, then the pooling
        (all-gather) or the replay exchange."""
        x = self.exchange if with_pool else None
        if x is not None:
            if not x.started:  # the replay buffer starts here: s of its first row = the current obs
                x.start(self.wl.envs[0].obs)
            x.before()
        p = self.pool if with_pool else None
        if p is not None and self.pool_every == SEG:
            p.begin()
        if p is not None and self.mode == "segment" and self.pool_every == SEG:
            buf = p.buf
        else:
            buf = None
        own = timed
        if timed:  # every event_every-th timed segment (the first always)
            own = own and self.timed_segments % self.event_every == 0
            self.timed_segments += 1
        if own:
            ea, eb = self._clock_pair()
            ea.record(self.st)
        if self.graphs is not None:
            gset = self.graphs[(k0 % ACTION_STEPS) // SEG]
            gset[p.buf if p is not None else 0].replay()
        else:
            self._steps(k0, with_pool, buf=buf, on_step=on_step, timed=timed)
        if own:
            eb.record(self.st)
            self.seg_events.append((ea, eb, SEG))
        if x is not None:
            x.launched()
        self.wl.refill()
        if p is not None and self.pool_every == SEG:
            p.fill = SEG
            p.flush()
        if x is not None:
            x.after()
        return k0 + SEG


# ---------------------------------------------------------------- timing loop
def _max_over_ranks(x: float, world: int, dev) -> float:
    if world <= 1:
        return x
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def make_exchange(args, wl: Workload, rank: int, world: int, dev, standin: dict | None = None):
    """The sharded pooling's replay exchange: a StagedReplay over this rank's envs (the
    pooled ReplayBuffer(--replay-mem) of every rank's envs, one learn() of
    --replay-batch per step; --sampler, --exchange) behind a SegmentExchange (its side
    stream). ``standin`` (N=1): the collective's kernel stood in for (StagedReplay)."""
    from sacenv.dist import SegmentExchange
    if args.stub:
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        from bench_stub import StubSampler
        sampler = StubSampler(wl.row_bytes(), SEG, args.replay_batch, world, exchange=args.exchange)
    else:
        from sacenv.replay import StagedReplay
        env = wl.envs[0]
        sampler = StagedReplay(env.num_envs, env.n_pad, args.experiment, env.first_obs_template(), rank=rank,
                               world=world, mem_size=args.replay_mem, batch=args.replay_batch, seg=SEG, seed=0,
                               device=dev, sampler=args.sampler, exchange=args.exchange, standin=standin)
    return SegmentExchange(sampler, dev)


def collective_standin(args, wl: Workload) -> dict:
    """The N=1 stand-in for the N>1 line's collective kernel: the bytes
    one rank moves per segment at --standin-world ranks (the all-gather's (W-1) chunks, or
    the ring all-reduce's 2 (W-1)/W payload), on --channels workgroups, resident for
    bytes / --standin-gbps."""
    W = max(2, int(args.standin_world))
    env = wl.envs[0]
    if args.exchange == "allgather":
        from sacenv.replay import staged_chunk
        _, chunk = staged_chunk(env.num_envs, env.n_pad, W, args.replay_mem, args.replay_batch, SEG,
                                args.experiment)
        nbytes = (W - 1) * chunk
    else:
        nbytes = 2 * (W - 1) / W * SEG * args.replay_batch * 26 * 4
    us = nbytes / (args.standin_gbps * 1e9) * 1e6
    return {"bytes": int(nbytes), "workgroups": int(args.channels), "us": us, "world": W}


def timed_rate(run: "SegmentRunner", k: int, n_segs: int, world: int, dev, wl: Workload):
    """One warm segment, then n_segs segments of ``run`` wall-timed between barriers
    (what they leave in flight included), max over ranks -> (rate dict, k, seconds)."""
    k = run.segment(k, False)
    run.finish()
    _sync(dev)
    barrier(world)
    _sync(dev)
    t0 = time.perf_counter()
    for _ in range(n_segs):
        k = run.segment(k, True)
    run.finish()
    _sync(dev)
    barrier(world)
    el = _max_over_ranks(time.perf_counter() - t0, world, dev)
    if run.exchange is not None:
        run.exchange.check()
    steps = n_segs * SEG
    return ({"value": world * wl.per_gpu_envs * steps / el, "unit": "env-steps/s", "steps": steps,
             "ms_per_step": el / steps * 1e3}, k, el)


def _xgmi(bytes_per_rank: float, seconds: float, links: int) -> dict:
    """Bytes a rank moves per second over its point-to-point xGMI links."""
    rate = bytes_per_rank / seconds / 1e9 if seconds > 0 else 0.0
    per_link = rate / max(1, links)
    return {"link_peak_GBps": XGMI_LINK_GBPS, "links_used": links, "GBps_per_rank": rate,
            "per_link_GBps": per_link, "per_link_frac": per_link / XGMI_LINK_GBPS}


def pooling_mode(args, world: int, wl: Workload) -> str:
    """The N>1 exchange this run can time: --pooling, except that the staged replay
    (sharded) needs the persistent segment launch -- it writes the staged rows -- and a
    boat-only workload; otherwise every transition is all-gathered (the
    sharded exchange under --launch step / --no-graph read rows no launch wrote). The
    CPU stub's sampler takes rows from any runner mode."""
    pooling = args.pooling if world > 1 else "none"
    if pooling == "sharded" and (args.mixed or not wl.segment_pools):
        return "gather"   # the toys of the mixed batch have no staged replay: their rows are gathered
    if pooling == "sharded" and not args.stub and (args.launch != "segment" or args.no_graph
                                                   or wl.segment_step is None):
        return "gather"
    return pooling


def run_bench(args, rank: int, world: int, dev, wl: Workload):
    """Warm up, time whole segments, measure the kernel; rank 0 returns the JSON dict.

    N>1 (``--pooling sharded``, the default): the segment launch stages the rows the
    pooled buffer's learns will read, each rank draws every learn (counter-based),
    packs its own sampled rows and ONE all-gather per segment (a side stream,
    overlapped with the next segment) gives every rank the segment's learn() batches
    -- inside the timed region. Beside it (after the timed region, same segments):
    the all-gather of every transition (configs[3]'s literal exchange) and no
    exchange at all. N=1: the replay path without a collective (``replay_path``),
    with the collective's kernel stood in for (``replay_path_collective_standin``)
    and this GPU as rank 0 of --standin-world ranks (``replay_path_rank_of_world``),
    so the per-GPU cost of the exchange is on the N=1 line."""
    pool_every = int(getattr(args, "pool_every", SEG))
    pooling = pooling_mode(args, world, wl)
    pool = exchange = None
    if pooling == "gather":
        from sacenv.dist import SegmentPool
        # each step's full transitions are written into row j of a [P][row] staging
        # buffer; ONE all-gather per P steps pools them on a side stream
        pool = SegmentPool(wl.row_bytes(), pool_every, dev)
    elif pooling == "sharded":
        exchange = make_exchange(args, wl, rank, world, dev)
        pool_every = SEG
    run = SegmentRunner(args, wl, dev, pool, pool_every, exchange)
    use_graph = run.use_graph
    run.prepare()
    st = run.st
    seg_events = run.seg_events
    segment = run.segment
    n_warm, n_timed = warm_segs(args.warmup), timed_segs(args.steps)
    if dev.type == "cuda":  # past the clock boost (~20 launches) before the rate is sized
        n_warm = max(n_warm, WARM_BOOST_SEGS)
    k = 0
    half = n_warm // 2
    t_w = time.perf_counter()
    for i in range(n_warm):
        if i == half:  # the rate of the warm-up's second half: after the boost
            run.finish()
            _sync(dev)
            t_w = time.perf_counter()
        k = segment(k, False)
    run.finish()
    _sync(dev)
    per_seg = (time.perf_counter() - t_w) / (n_warm - half)
    if dev.type == "cuda":  # (CPU stub runs measure the harness: no minimum duration)
        want = math.ceil(args.min_seconds * TIMED_MARGIN / max(per_seg, 1e-6))
        n_timed = int(_max_over_ranks(float(max(n_timed, want)), world, dev))
    barrier(world)
    _sync(dev)
    ev0, ev1 = _Clock(dev), _Clock(dev)
    run.reserve_clocks(2 * n_timed)
    t0 = time.perf_counter()
    ev0.record(st)
    g0 = pool.flushes if pool is not None else 0
    x0 = exchange.exchanges if exchange is not None else 0
    for _ in range(n_timed):
        k = segment(k, True)
    run.finish()  # the last segment's all-gather / exchange and the last refills are inside the timed region
    ev1.record(st)
    gathers_timed = (pool.flushes if pool is not None else 0) - g0
    exchanges_timed = (exchange.exchanges if exchange is not None else 0) - x0
    _sync(dev)
    barrier(world)
    el = time.perf_counter() - t0
    steps = n_timed * SEG
    el_max = _max_over_ranks(el, world, dev)
    if exchange is not None:  # (after the timed region: it synchronises)
        exchange.check()

    # the kernel's average launch duration from events on the stream it runs on,
    # refills excluded. N=1: the launches of the timed region itself. N>1 (the
    # segments also write the exchanged rows) or eager: launches after the timed
    # region with no exchange.
    what = ("persistent sacenv_boat_segment launches" if run.mode == "segment" else
            f"graph-replayed {SEG}-launch k_step segments")
    no_exchange = all_gather = None
    if pool is not None or exchange is not None or run.mode == "eager":
        if run.mode == "eager" and dev.type == "cuda" and not args.no_graph:
            run.capture_all(with_pool=False)
            run.mode, use_graph = "graph", True
            what = f"graph-replayed {SEG}-launch k_step segments"
        seg_events.clear()
        run.timed_segments = 0  # (the event stride restarts: the first of these is timed)
        k = segment(k, False, with_pool=False)
        # (N>1) the same segments and refills with no exchange, wall-timed like the
        # timed region: N x the one-GPU rate, reported beside
        n_ne = segs(args.kernel_launches)
        _sync(dev)
        barrier(world)
        _sync(dev)
        t_ne = time.perf_counter()
        for _ in range(n_ne):
            k = segment(k, True, with_pool=False)
        _sync(dev)
        barrier(world)
        el_ne = _max_over_ranks(time.perf_counter() - t_ne, world, dev)
        no_exchange = {"value": world * wl.per_gpu_envs * n_ne * SEG / el_ne, "steps": n_ne * SEG,
                       "ms_per_step": el_ne / (n_ne * SEG) * 1e3,
                       "note": "the same persistent segments and refills after the timed region with no exchange "
                               "(each rank's transitions stay on its GPU, nothing sampled), wall-timed between "
                               "barriers, max over ranks"}
        kern_src = (f"events around {len(seg_events)} {what if dev.type == 'cuda' else 'eager'} after the "
                    "timed region (no rows, no collective; refills between segments excluded)")
        if exchange is not None:
            # beside it: configs[3]'s literal exchange, every transition all-gathered per segment
            from sacenv.dist import SegmentPool
            gpool = SegmentPool(wl.row_bytes(), SEG, dev)
            grun = SegmentRunner(args, wl, dev, gpool, SEG)
            if grun.mode == "graph":        # (no captured graphs for this side run)
                grun.mode, grun.use_graph = "eager", False
            rate, k, el_g = timed_rate(grun, k, max(1, args.exchange_segs), world, dev, wl)
            recv = (world - 1) * wl.row_bytes() * rate["steps"]
            all_gather = dict(rate, gathers=gpool.flushes - 1, row_bytes_per_rank_step=wl.row_bytes(),
                              received_bytes_per_rank=recv, xgmi=_xgmi(recv, el_g, world - 1),
                              note=f"each segment's {TRANS_ROW} of every rank all-gathered (one "
                                   f"all_gather_into_tensor per {SEG}-step segment on a side stream, overlapped "
                                   "with the next segment), after the timed region, wall-timed, max over ranks")
    else:
        kern_src = (f"HIP events around the {len(seg_events)} {what} of the timed region (refills "
                    "between segments excluded)")
    kern_s = sum(a.ms_to(b) for a, b, _ in seg_events) * 1e-3 / sum(n for _, _, n in seg_events)
    step_s = ev0.ms_to(ev1) * 1e-3 / steps

    every = replay_path = standin_path = rank_path = None
    if (world == 1 and run.mode == "segment" and not args.mixed and not args.no_autoreset
            and not args.no_every_output):
        every = every_output_rate(wl, dev, k0=k)
    if world == 1 and not args.mixed and not args.no_autoreset and not args.no_every_output and (
            run.mode == "segment" or args.stub):
        # the sharded pooling's replay path on one GPU (no collective): rows staged, the
        # segment's learns sampled on a side stream overlapped with the next segment
        n_x = max(1, args.exchange_segs)
        xrun = SegmentRunner(args, wl, dev, None, SEG, make_exchange(args, wl, rank, 1, dev))
        rate, k, _ = timed_rate(xrun, k, n_x, world, dev, wl)
        replay_path = dict(rate, sampler=args.sampler, exchange=args.exchange, note=(
            f"the N>1 line's replay path at one GPU (--pooling sharded without the collective): each "
            f"segment's {SEG} learn() batches of {args.replay_batch} drawn ahead ("
            + ("counter-based: Philox4x64-10, np.random.choice's distribution per learn, one parallel "
               "launch that also marks the rows" if args.sampler == "philox" else
               "the pooled buffer's MT19937 stream, exact") +
            f") from the pooled ReplayBuffer({args.replay_mem}), the segment launch writing the 64-B rows they "
            "read, the batches " + ("packed per rank and unpacked (the all-gather's two roles; with the "
                                    "draws, one side launch per segment)"
                                    if args.exchange == "allgather" else "gathered") +
            " on the stepping stream after each segment's refill (sacenv.dist.SegmentExchange: kernels beside a "
            "launch or a refill slowed them more than they overlapped), after the timed region, wall time"))
        if not args.stub:
            sd = collective_standin(args, wl)
            srun = SegmentRunner(args, wl, dev, None, SEG, make_exchange(args, wl, rank, 1, dev, standin=sd))
            rate, k, _ = timed_rate(srun, k, n_x, world, dev, wl)
            standin_path = dict(rate, standin=sd, frac_of_replay_path=rate["value"] / replay_path["value"], note=(
                f"replay_path with the collective's kernel stood in for: between the pack and the unpack, "
                f"{sd['workgroups']} workgroups (the RCCL channel cap the N>1 line sets, NCCL_MAX_NCHANNELS) copy "
                f"the {sd['bytes']} B one rank moves per segment at {sd['world']} ranks and stay resident for "
                f"{sd['us']:.1f} us (those bytes at {args.standin_gbps:g} GB/s per rank), on a side stream "
                "beside the next segment's launch, as the N>1 collective runs; the unpack waits for it; no xGMI "
                "traffic"))
            if args.sampler == "philox" and args.exchange == "allgather":
                W = max(2, int(args.standin_world))
                rrun = SegmentRunner(args, wl, dev, None, SEG, make_exchange(args, wl, rank, W, dev, standin=sd))
                rate, k, _ = timed_rate(rrun, k, n_x, world, dev, wl)
                rank_path = dict(rate, world=W, standin=sd, note=(
                    f"this GPU's {wl.per_gpu_envs} envs as rank 0 of a {W}-rank pooled buffer (period {W} x "
                    f"{wl.per_gpu_envs}: the N = {W} line's per-rank work at one GPU): the draws of every learn, "
                    "the marks, staged rows and packed chunk of its own rows, the collective stood in for as "
                    "above (its own chunk copied into the gathered buffer, resident for the other ranks' "
                    f"{W - 1} chunks at {args.standin_gbps:g} GB/s), the unpack of all {W} chunks; the other "
                    "ranks' chunks were packed once, before the timed segments, from this GPU's rows under "
                    "their env ids (their slots and counts, not their transitions: timing only)"))
    dinfo = dist_info(world, dev)
    if rank != 0:
        return None
    seg_mode = run.mode == "segment"
    # the persistent launch keeps the carried state (152 of SURVEY §8(d)'s 222 B) in
    # registers between its steps: its algorithmic bytes are the same components
    # with the state read and written once per 256-step launch
    N = wl.envs[0].num_envs
    algo_step = SEG_MIN_BYTES * N if seg_mode else wl.bytes_per_launch
    if seg_mode and args.mixed:  # + the toys with their state resident: record 14 B per step
        algo_step += sum(TOY_SEG_BYTES.values()) * N
    achieved = algo_step / kern_s
    traffic = None if args.mixed or args.stub else load_traffic(N, args.experiment, "segment" if seg_mode else "step")
    compute = load_compute(N, args.experiment, kern_s) if seg_mode and not args.mixed and not args.stub else None
    if compute is not None and world > 1:
        compute["note"] += f" (PMC from the one-GPU run in {compute['source']}, applied to this run's kernel time)"
    backend = None
    if world > 1:
        import torch.distributed as dist
        backend = "RCCL" if dist.get_backend() == "nccl" else dist.get_backend()
    if exchange is not None:
        payload = exchange.sampler.bytes_per_segment
        what_x = (f"{backend} all_gather of each rank's packed rows of each {SEG}-step segment's {SEG} learn() "
                  f"batches ({args.replay_batch} rows; {payload} B gathered: 100-B records with their slot, "
                  "unpacked into the batches on every rank)" if args.exchange == "allgather" else
                  f"{backend} SUM all_reduce of each {SEG}-step segment's {SEG} learn() batches ({args.replay_batch} "
                  f"rows, {payload} B)")
        collective = (f"{what_x} of the pooled ReplayBuffer({args.replay_mem}) of every rank's envs, "
                      "gathered from the rows each rank's segment launch staged (sacenv.replay.StagedReplay: the "
                      "index draws made ahead, only the rows they read written; "
                      + ("counter-based draws (Philox4x64-10, np.random.choice's distribution per learn)"
                         if args.sampler == "philox" else "the reference stream's exact draws (MT19937)") +
                      f"): one per segment on a side stream, overlapped with the next segment "
                      f"({exchanges_timed} in the timed region)")
    elif pool is not None:
        collective = (f"all_gather of each step's full transitions (the {TRANS_ROW} written by the step kernel, "
                      f"{wl.row_bytes()} B per rank-step): one {backend} all_gather per {pool_every}-step "
                      + ("segment" if pool_every == SEG else "group") +
                      f" ({gathers_timed} in the timed region) on a side stream"
                      + (", overlapped with the next segment" if pool_every == SEG else ""))
    else:
        collective = "none: no exchange (--pooling none)" if world > 1 else None
    pooling_out = None
    if world > 1:
        pooling_out = {"mode": pooling, "no_exchange": no_exchange}
        if exchange is not None:
            payload = exchange.sampler.bytes_per_segment
            bus = exchange.sampler.bus_bytes_per_segment * exchanges_timed  # a ring schedule's bytes per rank
            pooling_out.update({
                "exchanges_timed": exchanges_timed, "bytes_per_segment": payload,
                "staged_row_bytes": 64, "sampler": args.sampler, "exchange": args.exchange,
                "bus_bytes_per_rank": bus, "xgmi": _xgmi(bus, el_max, world - 1),
                "all_gather": all_gather,
                "note": "value = the timed region with this exchange; all_gather and no_exchange are the same "
                        "segments with the other exchanges, after the timed region"})
        elif pool is not None:
            recv = (world - 1) * wl.row_bytes() * steps
            pooling_out.update({
                "pool_every": pool_every, "gathers_timed": gathers_timed,
                "row_bytes_per_rank_step": wl.row_bytes(), "received_bytes_per_rank": recv,
                "received_GBps_per_rank": recv / el_max / 1e9,
                # each peer's rows arrive over its own point-to-point link
                "xgmi": _xgmi(recv, el_max, world - 1),
                "note": "the timed region ends when the last all_gather has landed"})
    for fld in (every, replay_path, rank_path):   # (fractions of the headline value)
        if fld is not None:
            fld["frac_of_value"] = fld["value"] / (world * wl.per_gpu_envs * steps / el_max)
    return {
        "metric": metric_name(args),
        "value": world * wl.per_gpu_envs * steps / el_max,
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": n_warm * SEG,
        "requested": {"steps": args.steps, "warmup": args.warmup,
                      "rule": f"rounded up to whole {SEG}-step segments (each ends with its refill); "
                              f"at least {MIN_TIMED_SEGS * SEG} timed and {MIN_WARMUP_SEGS * SEG} warm-up steps, "
                              f"and timed segments for at least ~{args.min_seconds:g} s at the warm-up's rate"},
        "setup": {"graph_first_replays": run.first_replays,
                  "note": "steps of the first pass over the action table (a captured graph's first "
                          "replay carries its device upload), run before the warm-up, untimed"},
        "ms_per_step": el_max / steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": ("stub: CPU control-flow rehearsal, no kernels (tools/bench_stub.py)" if args.stub else
                 "synthetic: U(-1,1) f32 actions, per-env MT19937 wind/start draws (seeds = global env id)"),
        "config": {"workload": (f"mixed batch in one launch: boat_env exp {args.experiment} + "
                                f"toy_parachute + toy_car, {N} envs each/GPU" if args.mixed else
                                f"boat_env exp {args.experiment}, {N} envs/GPU") +
                               f", {args.episode_steps}-step episodes, in-kernel auto-reset" +
                               (f", pooled replay exchange per {SEG}-step segment" if exchange is not None else ""),
                   "experiment": args.experiment, "envs_per_gpu": wl.per_gpu_envs,
                   "global_envs": world * wl.per_gpu_envs,
                   "episode_steps": args.episode_steps, "parallelism": f"env-dp{world}",
                   "collective": collective,
                   "launch": ((f"one persistent sacenv_mixed_segment launch per {SEG} steps (the boat's owner "
                               "waves and every toy wave, state in registers)" if args.mixed else
                               f"one persistent sacenv_boat_segment launch per {SEG} steps") +
                              " (k_rollout: the carried state in registers; each owner wave checks its "
                              "action-row flag, all rows published) + the 3 refill launches after each"
                              + (f"; one launch per {pool_every} steps when pooling" if pool is not None
                                 and pool_every < SEG else "")
                              + ("; the launch writes each step's transition rows into the staged replay buffer"
                                 if exchange is not None else "")
                              if seg_mode else
                              (f"hipGraph segments of {SEG} k_step launches" +
                               (" (sacenv_boat_step_pooled: the step writes its pooled row)"
                                if pool is not None and not args.mixed else
                                " (+ the pooled-row copies per step)" if pool is not None else "") +
                               " + the 3 refill launches" if use_graph else "eager")),
                   "refill": None if args.no_autoreset else (
                       f"k_need_masks + k_refill + k_refill_fit after every {SEG}-step segment, inside the "
                       "timed region")},
        "roofline": {"bound": "fp64-issue" if compute is not None else "hbm",
                     "achieved": compute["achieved"] if compute is not None else achieved / 1e9,
                     "peak": compute["peak"] if compute is not None else HBM_PEAK / 1e9,
                     "unit": "TFLOP/s" if compute is not None else "GB/s",
                     "frac": compute["frac"] if compute is not None else achieved / HBM_PEAK,
                     "issue_floor_frac": None if compute is None else compute["issue_floor_frac"],
                     "limiter": ("FP64 VALU instruction issue of one owner wave per SIMD: achieved FP64 flop/s "
                                 "against the 78.6-TF FP64 vector datasheet peak; issue_floor_frac = the issue "
                                 "floor of the measured instruction stream / the kernel's time (compute); the "
                                 "byte rates and the PMC traffic are under hbm"
                                 if compute is not None else
                                 "launch + latency chains (DESIGN.md §4.2)" if not seg_mode else
                                 "instruction issue (no committed PMC pass for this shape)"),
                     "compute": compute,
                     "hbm": {"achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                             "frac": achieved / HBM_PEAK,
                             "traffic_frac": (None if traffic is None else
                                              traffic["hbm_bytes_per_launch"] / kern_s / HBM_PEAK)},
                     "traffic": None if traffic is None else traffic["hbm_bytes_per_launch"],
                     "kernel": ("k_rollout_mixed (sacenv_mixed_segment, 256 steps per launch; per step below)"
                                if seg_mode and args.mixed else
                                "k_rollout (sacenv_boat_segment, 256 steps per launch; per step below)"
                                if seg_mode else "k_step<true> (mixed)" if args.mixed else "k_step"),
                     "bytes_per_step": algo_step,
                     "bytes_per_env_step": (dict(boat=SEG_MIN_BYTES, **TOY_SEG_BYTES) if seg_mode and args.mixed
                                            else SEG_MIN_BYTES if seg_mode else
                                            dict(boat=BYTES_PER_ENV_STEP, **TOY_BYTES)
                                            if args.mixed else BYTES_PER_ENV_STEP),
                     "kernel_avg_us": kern_s * 1e6,
                     "step_us_incl_refill": step_s * 1e6,
                     "timing": kern_src,
                     "traffic_source": None if traffic is None else traffic["source"],
                     "algorithmic_bytes": (
                         "SURVEY §8(d)'s per-step components with the state resident: action 4 + wind "
                         "sample 16 + obs 44 + reward 4 + done/term 2 per env-step, state r+w 152 once "
                         "per 256-step launch" if seg_mode else "SURVEY §8(d): 222 B per boat env-step"),
                     # SURVEY §8(d)'s per-step contract (the state re-read and re-written every
                     # step, as a step launch must): the equivalent rate of the persistent launch
                     "survey_222B": None if not seg_mode else {
                         "bytes_per_env_step": BYTES_PER_ENV_STEP,
                         "equivalent_GBps": BYTES_PER_ENV_STEP * N / kern_s / 1e9,
                         "ratio_to_hbm_peak": BYTES_PER_ENV_STEP * N / kern_s / HBM_PEAK,
                         "note": "above 1: a step-per-launch design moving 222 B per env-step could not "
                                 "reach this rate at 8 TB/s; the persistent launch is bound by its "
                                 "instruction issue (one owner wave per SIMD), not by HBM"}},
        "every_output": every,
        "replay_path": replay_path,
        "replay_path_collective_standin": standin_path,
        "replay_path_rank_of_world": rank_path,
        "cpu_baseline": None,
        "dist": dinfo,
        "pooling": pooling_out,
    }


# ---------------------------------------------------------------- every-output rate
def every_output_rate(wl: Workload, dev, n_segs: int = 4, k0: int = 0) -> dict | None:
    """The same engine with EVERY step's outputs landing in HBM: K = SEG-step
    sacenv_boat_rollout launches writing each step's 50-B record (obs, reward, done,
    term) and terminal obs to their own rows (the persistent segment rewrites one
    record in place, so all but the last step's rows stay in L2), each followed by the
    refill; wall-timed between synchronizes."""
    if dev.type != "cuda":
        return None
    env, actions = wl.envs[0], wl.actions
    recs = torch.empty((SEG, 50 * env.n_pad), dtype=torch.uint8, device=dev)
    fin = torch.empty((SEG, env.n_pad, 11), dtype=torch.float32, device=dev)
    k = k0
    for _ in range(2):                       # warm (first launch of this instantiation)
        env.rollout(actions[k % ACTION_STEPS: k % ACTION_STEPS + SEG], recs, fin)
        env.refill()
        k += SEG
    _sync(dev)
    t0 = time.perf_counter()
    for _ in range(n_segs):
        env.rollout(actions[k % ACTION_STEPS: k % ACTION_STEPS + SEG], recs, fin)
        env.refill()
        k += SEG
    _sync(dev)
    el = time.perf_counter() - t0
    steps = n_segs * SEG
    return {"value": env.num_envs * steps / el, "unit": "env-steps/s", "steps": steps,
            "ms_per_step": el / steps * 1e3,
            "note": f"sacenv_boat_rollout, {SEG} steps per launch, every step's record and terminal obs "
                    "written to its own rows, + the refill per launch; after the timed region, wall time"}


# ---------------------------------------------------------------- closed-loop line
def bench_closed_loop(args, rank, world, dev):
    """main.py:70-91's acting loop on the device: every step the
    policy (NativeSAC choose_action: continuous_agent.py:57-61 on networks.py's actor,
    hand-written MFMA) reads the env's obs and writes the actions the env step reads,
    handing off per owner wave through device flags (sacenv.closed_loop.ClosedLoop): the
    env as persistent sacenv_boat_segment launches, the policy as one launch per step
    on a second stream, no host synchronisation between steps; the slot refill after
    each 256-step segment. Timed beside it: the same loop as main.py orders it
    (ClosedLoop.run_eager: choose_action then one step launch, one stream), which wins
    when the policy dominates the step; ``value`` is the faster form, ``modes`` both.
    The policy's noise comes from two pre-drawn [256, N] normal tables (the reference
    draws it inside choose_action)."""
    from sacenv import VecBoatEnv
    from sacenv.closed_loop import ClosedLoop
    from sacenv.sac_native import NativeSAC
    N = args.envs
    env = VecBoatEnv({"base_settings": {"experiment": args.experiment, "test_mode": args.test_mode}}, N,
                     seed=0, device=dev, max_episode_steps=args.episode_steps, env_id_offset=rank * N,
                     n_helpers=args.helpers, auto_refill=False)
    env.reset()
    agent = NativeSAC(dev, init_seed=rank, with_memory=False)
    loop = ClosedLoop(env, agent, segment=SEG, handoff=True)
    g = torch.Generator(device=dev)
    g.manual_seed(77 + rank)
    eps = torch.randn((2, SEG, N), generator=g, device=dev)
    state = {"i": 0}

    def segment(mode):
        e = eps[state["i"] % 2]
        loop.run_handoff(e) if mode == "handoff" else loop.run_eager(e)
        env.refill()
        state["i"] += 1

    n_timed = timed_segs(args.steps)
    steps = n_timed * SEG
    rates = {}
    # both forms of the loop (the same results, bit for bit: tests/test_segment_gpu.py),
    # each warmed up and timed over the same number of segments
    for mode in ("handoff", "eager"):
        for _ in range(warm_segs(args.warmup)):
            segment(mode)
        _sync(dev)
        loop.check()
        barrier(world)
        t0 = time.perf_counter()
        for _ in range(n_timed):
            segment(mode)
        _sync(dev)
        barrier(world)
        el = time.perf_counter() - t0
        loop.check()
        if world > 1:
            import torch.distributed as dist
            t = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        rates[mode] = {"value": world * N * steps / el, "unit": "env-steps/s", "ms_per_step": el / steps * 1e3}
    best = max(rates, key=lambda m: rates[m]["value"])
    el_max = rates[best]["ms_per_step"] * steps / 1e3
    # the policy alone (sacenv_sac_act on the env's obs, one launch per step) for the split
    ea, eb = _Clock(dev), _Clock(dev)
    st = torch.cuda.current_stream(dev)
    out = torch.empty(N, device=dev)
    agent.choose_action(env.obs, eps=eps[0, 0])
    ea.record(st)
    for k in range(32):
        agent.choose_action(env.obs, eps=eps[0, k])
    eb.record(st)
    _sync(dev)
    act_us = ea.ms_to(eb) * 1e3 / 32
    del out
    if rank != 0:
        return None
    return {
        "metric": f"env-steps/sec (whole node), boat_env exp-{args.experiment} closed loop (SAC actor + env "
                  f"step per step, device hand-off), {N:,} envs/GPU".replace(",", " "),
        "value": world * N * steps / el_max, "unit": "env-steps/s", "n_gpus": world, "steps": steps,
        "warmup": warm_segs(args.warmup) * SEG, "ms_per_step": el_max / steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64 env, f32 policy",
        "data": "synthetic: random-init actor (torch.manual_seed), N(0,1) policy noise tables, per-env MT19937 "
                "wind/start draws",
        "config": {"workload": f"boat_env exp {args.experiment}, {N} envs/GPU, {args.episode_steps}-step "
                               "episodes, in-kernel auto-reset; policy: NativeSAC choose_action (256-256 actor, "
                               "tanh-squashed Normal) per step",
                   "envs_per_gpu": N, "parallelism": f"env-dp{world}",
                   "launch": {"handoff": "one persistent sacenv_boat_segment launch per 256 steps "
                                         "(act_ready / step_done flags per owner wave) + one "
                                         "sacenv_sac_act_handoff launch per step on a second stream + the 3 "
                                         "refill launches per segment",
                              "eager": "per step one sacenv_sac_act launch then one sacenv_boat_step launch "
                                       "(main.py:78-81's order, one stream) + the 3 refill launches per segment"},
                   "value_mode": best,
                   "co_residency": {k: getattr(loop.plan, k) for k in ("seg_vgprs", "act_vgprs", "act_lds",
                                                                       "owner_waves_per_simd", "max_envs")}},
        "modes": rates,
        "policy_alone_us_per_step": act_us,
        "cpu_baseline": None}


# ---------------------------------------------------------------- training-loop line
def bench_train(args, rank, world, dev):
    """main.py:78-90's loop, every step, for every env of the rank at once:
    NativeSAC choose_action on the [N, 11] obs (continuous_agent.py:57-61, one MFMA launch),
    VecBoatEnv.step (one launch, auto-reset in-kernel; the slot refill every 256 steps),
    DeviceReplayBuffer.store_env_step (agent/buffer.py:13-22 with main.py:83-88's terminal:
    one launch for the N transitions), then one learn() (continuous_agent.py:96-154:
    sample_buffer(1 024) on the device + the four losses and Adam steps on MFMA kernels).
    The policy noise of choose_action and learn comes from pre-drawn tables (the reference
    draws it inside). Beside the loop's rate: each part timed alone with HIP events."""
    from sacenv import VecBoatEnv
    from sacenv.sac_native import NativeSAC
    N = args.envs
    env = VecBoatEnv({"base_settings": {"experiment": args.experiment, "test_mode": args.test_mode}}, N,
                     seed=0, device=dev, max_episode_steps=args.episode_steps, env_id_offset=rank * N,
                     n_helpers=args.helpers)
    env.reset()
    agent = NativeSAC(dev, init_seed=rank)
    B = agent.cfg.batch_size
    g = torch.Generator(device=dev)
    g.manual_seed(99 + rank)
    eps = torch.randn((SEG, N), generator=g, device=dev)
    noise = torch.randn((SEG, 2, B), generator=g, device=dev)
    prev = torch.empty_like(env.obs)
    counts = {"learns": 0}

    def step(k):
        prev.copy_(env.obs)
        a = agent.choose_action(env.obs, eps=eps[k % SEG])
        env.step_async(a.view(-1))
        agent.memory.store_env_step(prev, a, env)
        if agent.learn(noise=(noise[k % SEG, 0], noise[k % SEG, 1]), losses=False) is not None:
            counts["learns"] += 1

    k = 0
    for _ in range(warm_segs(args.warmup) * SEG):
        step(k)
        k += 1
    _sync(dev)
    barrier(world)
    n_timed = timed_segs(args.steps)
    steps = n_timed * SEG
    l0 = counts["learns"]
    t0 = time.perf_counter()
    for _ in range(steps):
        step(k)
        k += 1
    _sync(dev)
    barrier(world)
    el = _max_over_ranks(time.perf_counter() - t0, world, dev)
    learns = counts["learns"] - l0
    env.check_status()

    # each part alone (HIP events on the stream they run on), 64 repetitions
    st = torch.cuda.current_stream(dev)

    def timed(fn, reps=64):
        fn()
        ea, eb = _Clock(dev), _Clock(dev)
        ea.record(st)
        for _ in range(reps):
            fn()
        eb.record(st)
        _sync(dev)
        return ea.ms_to(eb) * 1e3 / reps

    a0 = agent.choose_action(env.obs, eps=eps[0]).view(-1).contiguous()
    parts = {"choose_action_us": timed(lambda: agent.choose_action(env.obs, eps=eps[0])),
             "env_step_us": timed(lambda: env.step_async(a0)),
             "store_us": timed(lambda: agent.memory.store_env_step(prev, a0, env)),
             "sample_us": timed(lambda: agent.memory.sample(B)),
             "learn_us": timed(lambda: agent.learn(noise=(noise[0, 0], noise[0, 1]), losses=False))}
    if rank != 0:
        return None
    return {
        "metric": f"env-steps/sec (whole node), boat_env exp-{args.experiment} training loop (act + step + store "
                  f"+ sample + learn per step), {N:,} envs/GPU".replace(",", " "),
        "value": world * N * steps / el, "unit": "env-steps/s", "n_gpus": world, "steps": steps,
        "warmup": warm_segs(args.warmup) * SEG, "ms_per_step": el / steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64 env, f32 agent",
        "data": "synthetic: random-init SAC networks (torch.manual_seed), N(0,1) policy noise tables, per-env "
                "MT19937 wind/start draws",
        "config": {"workload": f"boat_env exp {args.experiment}, {N} envs/GPU, {args.episode_steps}-step episodes, "
                               f"in-kernel auto-reset; NativeSAC (256-256 MLPs, batch {B}, ReplayBuffer"
                               f"({agent.memory.mem_size})), one learn() per step",
                   "envs_per_gpu": N, "parallelism": f"env-dp{world}" + (" (independent replicas)" if world > 1
                                                                          else ""),
                   "launch": "per step: sacenv_sac_act, sacenv_boat_step, sacenv_replay_store_env, "
                             "sacenv_replay_sample (draw + gather), sacenv_sac_learn (4 launches); the slot refill "
                             "every 256 steps"},
        "learns_timed": learns,
        "parts": parts,
        "note": "the loop is learn-bound: one learn() of a 1 024-row batch per step of all N envs (the "
                "reference's ratio is one learn per env step of ONE env)",
        "cpu_baseline": None}


# ---------------------------------------------------------------- rollout line
def bench_rollout(args, wl: Workload, rank, world, dev):
    """SURVEY.md §7.6 K-step fused rollout: K steps of an open-loop action sequence per
    launch (state in registers), every step's record (+ terminal obs) written out."""
    env, actions = wl.envs[0], wl.actions
    K = args.rollout
    if SEG % K:
        raise SystemExit(f"--rollout K must divide {SEG}")
    N = env.num_envs
    recs = torch.empty((K, 50 * env.n_pad), dtype=torch.uint8, device=dev)
    fin = torch.empty((K, env.n_pad, 11), dtype=torch.float32, device=dev)
    st = torch.cuda.current_stream(dev)
    seg_events = []

    def run(n_segs, k, timed=False):
        for _ in range(n_segs):
            for _ in range(SEG // K):
                if timed:
                    ea, eb = _Clock(dev), _Clock(dev)
                    ea.record(st)
                env.rollout(actions[k % ACTION_STEPS: k % ACTION_STEPS + K], recs, fin)
                if timed:
                    eb.record(st)
                    seg_events.append((ea, eb))
                k += K
            env.refill()
        return k

    k = run(warm_segs(args.warmup), 0)
    _sync(dev)
    barrier(world)
    n_timed = segs(args.steps)
    t0 = time.perf_counter()
    run(n_timed, k, timed=True)
    _sync(dev)
    barrier(world)
    el = time.perf_counter() - t0
    steps = n_timed * SEG
    el_max = el
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el_max = float(t.item())
    kern_s = sum(a.ms_to(b) for a, b in seg_events) * 1e-3 / (K * len(seg_events))
    bytes_env = 4 + 50 + 152 / K
    if rank != 0:
        return None
    return {
        "metric": f"env-steps/sec (whole node), boat_env exp-{args.experiment} open-loop K-step rollout, "
                  f"{N} envs/GPU",
        "value": world * N * steps / el_max, "unit": "env-steps/s", "n_gpus": world,
        "steps": steps, "warmup": warm_segs(args.warmup) * SEG, "ms_per_step": el_max / steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic: U(-1,1) f32 actions, per-env MT19937 wind/start draws",
        "config": {"workload": f"boat_env exp {args.experiment}, {N} envs/GPU, open-loop actions, "
                               f"{K} steps per sacenv_boat_rollout launch, every step's record "
                               f"and terminal obs written, refill every {SEG} steps",
                   "rollout_k": K, "envs_per_gpu": N, "parallelism": f"env-dp{world}"},
        "roofline": {"bound": "hbm", "achieved": bytes_env * N / kern_s / 1e9, "peak": HBM_PEAK / 1e9,
                     "unit": "GB/s", "frac": bytes_env * N / kern_s / HBM_PEAK,
                     "bytes_per_env_step": bytes_env, "kernel": "k_rollout",
                     "kernel_avg_us_per_step": kern_s * 1e6, "traffic": None,
                     "note": "algorithmic bytes: action 4 + record 50 per step, state r+w 152 per K"},
        "cpu_baseline": None}


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher: start the N rank processes here (before anything touches a GPU)
        sys.exit(spawn_ranks(args.gpus, argv))
    cpu = None
    if (int(os.environ.get("WORLD_SIZE", "1")) == 1 and not args.no_cpu_baseline and not args.rollout
            and not args.closed_loop and not args.train and not args.stub):
        # before anything touches the GPU: the C1 legs are child processes, and an
        # idle host keeps them from competing with the timed region's launches
        cpu = cpu_baseline(args, args.mixed_envs if args.mixed else args.envs)
    rank, world, dev = init_dist(args.gpus, args.stub, args.channels)
    if args.stub:
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import bench_stub
        _, wl = bench_stub.workload(sys.modules[__name__], rank)
        out = run_bench(args, rank, world, dev, wl)
        if out is not None:
            print(json.dumps(out), flush=True)
        if world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
        return
    if args.closed_loop or args.train:
        out = (bench_closed_loop if args.closed_loop else bench_train)(args, rank, world, dev)
        if out is not None:
            print(json.dumps(out), flush=True)
        if world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
        return
    wl = make_workload(args, rank, dev)
    if args.rollout:
        out = bench_rollout(args, wl, rank, world, dev)
    else:
        out = run_bench(args, rank, world, dev, wl)
    if out is not None and cpu is not None:
        out["cpu_baseline"] = cpu
    if out is not None:
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
