"""Benchmark: env-steps/s of the HIP boat env (BASELINE.json metric).

Workload (BASELINE.json configs[2] at N=1, configs[3] at N>1): boat_env
experiment 6 (random wind in all directions), 65 536 envs per GPU,
test_mode 0 (actions drive the rudder), actions U(-1,1) f32 pre-generated as
a [500, N] table in HBM, episodes truncated at 500 steps and auto-reset in
the step kernel (early terminations too). One "step" = one BoatEnv.step
over all envs of the rank (+ at N>1 the packed (obs, reward, done, term)
all-gather over RCCL that pools transitions for a shared replay buffer).

    python bench.py [--gpus N] [--steps K] [--warmup W]

Timing: W untimed steps, then exactly K steps bracketed by barrier +
synchronize; value = all envs x K / max-over-ranks time. Every 128 steps the
slot refill (k_refill: the RNG draws and spline fits of the episodes that
replace the ended ones) runs as its own launch INSIDE the timed region. At
N=1 the 128-step segments are replayed from hipGraphs (launch-bound
otherwise). Roofline: SURVEY.md §8(d) algorithmic 222 B per boat env-step x
envs per launch, over k_step's average launch duration from HIP events on
the kernel's stream around the 128-launch segments of the timed region (the
refills in between excluded; they are in ms_per_step); `traffic` = HBM bytes
per launch from the committed rocprofv3 PMC passes (tools/pmc.sh).
cpu_baseline: the numpy float64 oracle (oracle/boat_oracle.py, a port of the
reference step) on the same workload shape, one core, bounded sample.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "sac-agent_amd"))

METRIC = "env-steps/sec (whole node), boat_env exp-6, 65 536 envs/GPU at 1/2/4/8 MI355X"
BYTES_PER_ENV_STEP = 222      # state r+w 152, action 4, wind 16, obs 44, reward 4, done+term 2
TOY_BYTES_PER_ENV_STEP = 86 + 102  # parachute 86 B, car 102 B
METRIC_MIXED = ("env-steps/sec (whole node), mixed batch boat_env exp-6 + toy_parachute + toy_car, "
                "32 768 envs each/GPU")
HBM_PEAK = 8.0e12             # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
EPISODE_STEPS = 500
SEG = 128              # step launches per refill (sacenv _lib.REFILL_PERIOD); one graph per segment
ACTION_STEPS = 512     # the pre-generated action table cycles every 512 steps (4 segments)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=500)
    ap.add_argument("--envs", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--experiment", type=int, default=6)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--kernel-launches", type=int, default=200)
    ap.add_argument("--test-mode", type=int, default=0, help="1 = rudder frozen (no terminations)")
    ap.add_argument("--helpers", type=int, default=8192, help="workgroups of a refill draw launch")
    ap.add_argument("--mixed", action="store_true",
                    help="BASELINE configs[4]: boat exp-6 + toy_parachute + toy_car in one launch")
    ap.add_argument("--mixed-envs", type=int, default=32768, help="envs per type per GPU (--mixed)")
    ap.add_argument("--no-autoreset", action="store_true",
                    help="diagnostic: no in-kernel auto-reset (ended envs keep stepping)")
    ap.add_argument("--rollout", type=int, default=0,
                    help="K > 0: open-loop K-step rollouts (sacenv_boat_rollout), a separate line")
    ap.add_argument("--pooling", choices=("gather", "none"), default="gather",
                    help="N>1: all-gather the records per 128-step segment (configs[3]), or none "
                         "(sharded per-GPU replay, SURVEY.md §8(e)'s alternative to measure)")
    ap.add_argument("--episode-steps", type=int, default=EPISODE_STEPS,
                    help="truncation length (0 = none)")
    return ap.parse_args()


def init_dist(n_gpus: int):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != n_gpus:
        raise SystemExit(f"--gpus {n_gpus} but WORLD_SIZE={world}: launch N>1 with torch.distributed.run")
    if os.environ.get("SACENV_BENCH_ONE_DEVICE"):  # rehearsal of the N>1 path on a 1-GPU box
        local = 0
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = os.environ.get("SACENV_BENCH_BACKEND", "nccl")  # gloo: rehearsal on one GPU
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, torch.device("cuda", local)


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def cpu_baseline(n_envs: int, seconds: float, experiment: int, mixed: bool = False) -> dict:
    """The oracles (numpy ports of BoatEnv.step and of the toy scripts) on the
    bench workload shape, 1 thread, bounded sample."""
    try:
        from threadpoolctl import threadpool_limits
    except Exception:  # noqa: BLE001
        threadpool_limits = None
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from boat_oracle import OracleConfig, OracleVecBoat

    import contextlib
    ctx = threadpool_limits(limits=1) if threadpool_limits else contextlib.nullcontext()
    with ctx:
        seeds = np.arange(n_envs, dtype=np.uint64)
        # the constructor builds every env's first Boat (boat_env.py:15), untimed
        ora = OracleVecBoat(OracleConfig(experiment=experiment, test_mode=0), seeds,
                            max_episode_steps=EPISODE_STEPS)
        toys = []
        if mixed:
            from toy_oracle import OracleToy
            toys = [OracleToy(k, n_envs, max_episode_steps=EPISODE_STEPS) for k in (1, 2)]
        acts = np.random.default_rng(0).uniform(-1, 1, (64, n_envs)).astype(np.float32)
        ora.step(acts[0])  # warm
        steps, t0 = 0, time.perf_counter()
        while True:
            ora.step(acts[steps % 64])
            for t in toys:
                t.step()
            steps += 1
            el = time.perf_counter() - t0
            if el >= seconds and steps >= 3:
                break
    n_total = n_envs * (1 + len(toys))
    what = "boat + parachute + car oracles" if mixed else "oracle/boat_oracle.py"
    return {"value": n_total * steps / el, "unit": "env-steps/s", "cores": 1, "kind": "port",
            "sample": f"{what} numpy f64, exp {experiment}, {n_total} envs x "
                      f"{steps} steps ({el:.1f} s), auto-reset + 500-step truncation, 1 thread",
            "note": "reference BoatEnv itself (pure Python, 1 env, 1 core) measured 12 584 "
                    "env-steps/s for exp 6 in the survey container (BASELINE.md)"}


def load_traffic(n_envs: int, experiment: int):
    """Per-launch HBM bytes of k_step from the committed rocprofv3 PMC summary
    (tools/pmc.sh -> profiles/<round>_pmc_k_step.json, newest round first) for
    this workload shape, or None."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_k_step.json")), reverse=True):
        try:
            d = json.load(open(path))
        except Exception:  # noqa: BLE001
            continue
        if int(d.get("envs", -1)) == n_envs and int(d.get("experiment", 6)) == experiment \
                and "hbm_bytes_per_launch" in d:
            return {"hbm_bytes_per_launch": float(d["hbm_bytes_per_launch"]),
                    "source": os.path.relpath(path, ROOT)}
    return None


def bench_rollout(args, env, actions, rank, world, dev):
    """SURVEY.md §7.6 K-step fused rollout: K steps of an open-loop action sequence per
    launch (state in registers), every step's record (+ terminal obs) written out."""
    K = args.rollout
    if SEG % K:
        raise SystemExit(f"--rollout K must divide {SEG}")
    N = env.num_envs
    recs = torch.empty((K, 50 * env.n_pad), dtype=torch.uint8, device=dev)
    fin = torch.empty((K, env.n_pad, 11), dtype=torch.float32, device=dev)
    st = torch.cuda.current_stream(dev)
    seg_events = []

    def run(n_steps, k, timed=False):
        done = 0
        while done < n_steps:
            if timed:
                ea, eb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                ea.record(st)
            env.rollout(actions[k % ACTION_STEPS: k % ACTION_STEPS + K], recs, fin)
            if timed:
                eb.record(st)
                seg_events.append((ea, eb))
            k += K
            done += K
            if k % SEG == 0:
                env.refill()
        return k

    k = run(args.warmup // SEG * SEG or SEG, 0)
    torch.cuda.synchronize(dev)
    barrier(world)
    steps = max(SEG, args.steps // SEG * SEG)
    t0 = time.perf_counter()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(st)
    run(steps, k, timed=True)
    ev1.record(st)
    torch.cuda.synchronize(dev)
    barrier(world)
    el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64, device=dev)
    if world > 1:
        import torch.distributed as dist
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el_max = float(t.item())
    kern_s = sum(a.elapsed_time(b) for a, b in seg_events) * 1e-3 / (K * len(seg_events))
    bytes_env = 4 + 50 + 152 / K
    if rank == 0:
        print(json.dumps({
            "metric": "env-steps/sec (whole node), boat_env exp-6 open-loop K-step rollout, "
                      "65 536 envs/GPU",
            "value": world * N * steps / el_max, "unit": "env-steps/s", "n_gpus": world,
            "steps": steps, "warmup": args.warmup, "ms_per_step": el_max / steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic: U(-1,1) f32 actions, per-env MT19937 wind/start draws",
            "config": {"workload": f"boat_env exp {args.experiment}, {N} envs/GPU, open-loop actions, "
                                   f"{K} steps per sacenv_boat_rollout launch, every step's record "
                                   f"and terminal obs written, refill every {SEG} steps",
                       "rollout_k": K, "envs_per_gpu": N, "parallelism": f"env-dp{world}"},
            "roofline": {"bound": "hbm", "achieved": bytes_env * N / kern_s / 1e9, "peak": HBM_PEAK / 1e9,
                         "unit": "GB/s", "frac": bytes_env * N / kern_s / HBM_PEAK,
                         "bytes_per_env_step": bytes_env, "kernel": "k_rollout",
                         "kernel_avg_us_per_step": kern_s * 1e6,
                         "note": "algorithmic bytes: action 4 + record 50 per step, state r+w 152 per K"},
            "cpu_baseline": None}), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def main():
    args = parse()
    rank, world, dev = init_dist(args.gpus)
    from sacenv import VecBoatEnv

    N = args.mixed_envs if args.mixed else args.envs
    env = VecBoatEnv({"base_settings": {"experiment": args.experiment, "test_mode": args.test_mode}},
                     N, seed=0, device=dev, autoreset=not args.no_autoreset,
                     max_episode_steps=args.episode_steps,
                     env_id_offset=rank * N, n_helpers=args.helpers, auto_refill=False)
    env.reset()
    from sacenv import _lib
    assert SEG == _lib.REFILL_PERIOD
    autoreset = not args.no_autoreset
    refill = env.refill if autoreset else (lambda: None)
    envs, stepper = [env], env.step_async
    if args.mixed:
        from sacenv.toys import CarEnv, MixedBatch, ParachuteEnv
        toys = [ParachuteEnv(num_envs=N, device=dev, max_episode_steps=args.episode_steps),
                CarEnv(num_envs=N, device=dev, max_episode_steps=args.episode_steps)]
        envs += toys
        stepper = MixedBatch(env, toys).step_async
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    actions = (torch.rand((ACTION_STEPS, N), generator=g, device=dev, dtype=torch.float32) * 2 - 1)
    pool = None
    if world > 1:
        import torch.distributed as dist
    if world > 1 and args.pooling == "gather":
        from sacenv.dist import SegmentPool
        # Pooling (obs, reward, done, term) for the shared replay buffer: each
        # step's packed records are copied into row j of a [SEG][record] staging
        # buffer (graph-captured with the steps) and ONE all-gather per segment
        # pools them on a side stream while the next segment steps (fewer,
        # larger collectives: 420 MB per rank at 65 536 envs).
        pool = SegmentPool(sum(e.record.numel() for e in envs), SEG, dev)
    pooling = {"on": pool is not None}

    def step_eager(k: int):
        stepper(actions[k % ACTION_STEPS])
        if pooling["on"]:
            pool.push([e.record for e in envs])  # flushes at the segment's end
        if (k + 1) % SEG == 0:
            refill()

    if args.rollout:
        return bench_rollout(args, env, actions, rank, world, dev)
    use_graph = not args.no_graph
    graphs = []

    def capture(k0: int, buf: int = -1) -> torch.cuda.CUDAGraph:
        gr = torch.cuda.CUDAGraph()
        # thread_local: a collective library thread querying its events while this
        # thread captures must not invalidate the capture
        with torch.cuda.graph(gr, capture_error_mode="thread_local"):
            for j, k in enumerate(range(k0, k0 + SEG)):
                stepper(actions[k % ACTION_STEPS])
                if buf >= 0:
                    pool.stage_row(j, [e.record for e in envs], buf)
        return gr

    if use_graph:
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            for k in range(3):
                step_eager(k)
        torch.cuda.current_stream(dev).wait_stream(s)
        if pool is not None:
            pool.fill = 0
        refill()
        torch.cuda.synchronize(dev)
        # N>1: one graph per (segment of the action table, staging buffer)
        graphs = [[capture(base, b) for b in ((0, 1) if world > 1 else (-1,))]
                  for base in range(0, ACTION_STEPS, SEG)]

    st = torch.cuda.current_stream(dev)
    seg_events = []

    def run(n_steps: int, k0: int, timed: bool = False) -> int:
        k = k0
        done = 0
        while done < n_steps:
            if use_graph and k % SEG == 0 and n_steps - done >= SEG:
                if pooling["on"]:
                    pool.begin()
                if timed:
                    ea, eb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    ea.record(st)
                gset = graphs[(k % ACTION_STEPS) // SEG]
                gset[pool.buf if pooling["on"] else 0].replay()
                if timed:
                    eb.record(st)
                    seg_events.append((ea, eb))
                refill()
                if pooling["on"]:
                    pool.fill = SEG
                    pool.flush()
                k += SEG
                done += SEG
            else:
                step_eager(k)
                k += 1
                done += 1
        if timed and pooling["on"]:
            pool.flush()  # a partial segment's records are pooled inside the timed region
        return k

    k = run(args.warmup, 0)
    torch.cuda.synchronize(dev)
    barrier(world)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(st)
    g0 = pool.flushes if pool is not None else 0
    k = run(args.steps, k, timed=True)
    gathers_timed = (pool.flushes if pool is not None else 0) - g0
    ev1.record(st)
    torch.cuda.synchronize(dev)
    barrier(world)
    el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el_max = float(t.item())

    # k_step average launch duration from HIP events on the stream the kernel
    # runs on, around 128-launch graph segments (refills excluded). N=1: the
    # segments of the timed region itself. N>1: the timed region also holds
    # the all-gathers, so k_step-only segments are replayed and timed after it.
    if world > 1 or not use_graph:
        k0 = (k + SEG - 1) // SEG * SEG
        while k < k0:  # align to a segment boundary (refill after the last eager step)
            step_eager(k)
            k += 1
        torch.cuda.synchronize(dev)
        pooling["on"] = False  # k_step alone: no staging copies, no collective
        graphs = [[capture(base)] for base in range(0, ACTION_STEPS, SEG)]
        use_graph = True
        seg_events.clear()
        run(SEG, k)
        torch.cuda.synchronize(dev)
        run(max(SEG, args.kernel_launches // SEG * SEG), k, timed=True)
        torch.cuda.synchronize(dev)
        kern_src = (f"HIP events around {len(seg_events)} graph-replayed {SEG}-launch k_step segments "
                    "after the timed region (no staging copy, no collective; refills between segments excluded)")
    else:
        kern_src = (f"HIP events around the {len(seg_events)} graph-replayed {SEG}-launch k_step "
                    "segments of the timed region (refills between segments excluded)")
    kern_s = sum(a.elapsed_time(b) for a, b in seg_events) * 1e-3 / (SEG * len(seg_events))
    step_s = ev0.elapsed_time(ev1) * 1e-3 / args.steps

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    per_gpu_envs = N * len(envs)
    bytes_env = BYTES_PER_ENV_STEP + (TOY_BYTES_PER_ENV_STEP if args.mixed else 0)
    bytes_launch = bytes_env * N
    achieved = bytes_launch / kern_s
    traffic = None if args.mixed else load_traffic(N, args.experiment)
    out = {
        "metric": METRIC_MIXED if args.mixed else METRIC,
        "value": world * per_gpu_envs * args.steps / el_max,
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": el_max / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic: U(-1,1) f32 actions, per-env MT19937 wind/start draws (seeds 0..N-1)",
        "config": {"workload": (f"mixed batch in one launch: boat_env exp {args.experiment} + "
                                f"toy_parachute + toy_car, {N} envs each/GPU" if args.mixed else
                                f"boat_env exp {args.experiment}, {N} envs/GPU") +
                               f", {EPISODE_STEPS}-step episodes, in-kernel auto-reset",
                   "experiment": args.experiment, "envs_per_gpu": per_gpu_envs,
                   "global_envs": world * per_gpu_envs,
                   "episode_steps": EPISODE_STEPS, "parallelism": f"env-dp{world}",
                   "collective": (f"all_gather of the (obs,reward,done,term) records, 50 B/env/step: "
                                  f"one {'RCCL' if dist.get_backend() == 'nccl' else dist.get_backend()} all_gather per {SEG}-step segment ({gathers_timed} in the "
                                  "timed region) on a side stream, overlapped with the next segment")
                   if pool is not None else (
                       "none: sharded per-GPU replay (--pooling none)" if world > 1 else None),
                   "launch": (f"hipGraph segments of {SEG} k_step launches" +
                              (" (+ a record copy into the pooling buffer per step)" if world > 1 else "") +
                              " + the 3 refill launches" if not args.no_graph else "eager"),
                   "refill": f"k_need_masks + k_refill + k_refill_fit every {SEG} steps, inside the timed region" if autoreset else None},
        "roofline": {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK,
                     "traffic": None if traffic is None else traffic["hbm_bytes_per_launch"],
                     "kernel": "k_step<true> (mixed)" if args.mixed else "k_step",
                     "bytes_per_launch": bytes_launch,
                     "bytes_per_env_step": ({"boat": BYTES_PER_ENV_STEP, "parachute": 86, "car": 102}
                                            if args.mixed else BYTES_PER_ENV_STEP),
                     "kernel_avg_us": kern_s * 1e6,
                     "step_us_incl_refill": step_s * 1e6,
                     "timing": kern_src,
                     "traffic_source": None if traffic is None else traffic["source"]},
        "cpu_baseline": None,
    }
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(N, args.cpu_seconds, args.experiment, args.mixed)
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
