"""the CPU restatement at N=1, one core and all cores.

C1 is the reference's own CPU-runnable case: one env per process.
* 1 core: the restatement with one env, pinned to one CPU (``os.sched_setaffinity``,
  the ``taskset -c 0`` of §8(d)). ``--mode scalar`` (default, SURVEY §7.2's "scalar
  N=1 mode"): oracle/boat_scalar.py, Python floats and ``math`` per step;
  ``--mode numpy``: oracle/boat_oracle.py vectorised over its one env (pays numpy's
  per-call cost on 1-element arrays; kept as a secondary figure).
* all cores: one such process per CPU of this process's affinity set (capped by
  ``--max-procs``: the GPU box gives a job 16 CPUs while ``nproc`` shows the host's).
Actions U(-1,1) float64 from ``np.random.default_rng(rank)``; auto-reset on done or
every 500 steps, as in §8(d). Each process runs for a fixed wall time. C1 is exp 1;
``--experiments 1,6`` adds the bench's experiment (exp 6 resets draw wind splines,
as the reference's do).

Test / measurement infrastructure: this imports the oracle and is never part of the
product path. Prints one JSON line.

    python tools/cpu_c1.py [--seconds 10] [--max-procs 16] [--experiments 1,6]
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(rank: int, cpu: int, seconds: float, experiment: int, mode: str, q) -> None:
    os.environ["OMP_NUM_THREADS"] = "1"
    try:
        os.sched_setaffinity(0, {cpu})
    except OSError:
        pass
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from boat_oracle import OracleConfig, OracleVecBoat
    cfg = OracleConfig(experiment=experiment, test_mode=0)
    rng = np.random.default_rng(rank)
    acts = rng.uniform(-1.0, 1.0, (4096, 1))
    if mode == "scalar":
        from boat_scalar import ScalarBoat
        boat = ScalarBoat(cfg, rank, max_episode_steps=500)
        boat.reset()
        acts = acts[:, 0].tolist()

        def step(a):  # main.py:70-91: reset when the episode ends (or is truncated at 500)
            if boat.step(a)[2]:
                boat.reset()
    else:
        ora = OracleVecBoat(cfg, [rank], max_episode_steps=500)
        ora.reset()
        step = ora.step
    step(acts[0])
    steps, t0 = 0, time.perf_counter()
    while True:
        for k in range(256):
            step(acts[(steps + k) % 4096])
        steps += 256
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    q.put((rank, steps, el))


def _leg(cpus, seconds, experiment, mode="scalar"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_run, args=(r, c, seconds, experiment, mode, q)) for r, c in enumerate(cpus)]
    for p in ps:
        p.start()
    res = [q.get(timeout=seconds * 10 + 120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    # whole-leg rate: every process's steps over the longest process's time
    return sum(s for _, s, _ in res) / max(e for _, _, e in res)


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--max-procs", type=int, default=16)
    ap.add_argument("--experiments", default="1")
    ap.add_argument("--mode", choices=("scalar", "numpy"), default="scalar")
    ap.add_argument("--numpy-one-core", action="store_true",
                    help="also time --mode numpy on one core (a secondary figure)")
    a = ap.parse_args(argv)
    cpus = sorted(os.sched_getaffinity(0))
    allc = cpus[:max(1, a.max_procs)]
    legs = {}
    for e in (int(x) for x in a.experiments.split(",")):
        legs[str(e)] = {"one_core": {"env_steps_per_s": _leg(cpus[:1], a.seconds, e, a.mode), "procs": 1},
                        "all_cores": {"env_steps_per_s": _leg(allc, a.seconds, e, a.mode),
                                      "procs": len(allc)}}
        if a.numpy_one_core and a.mode != "numpy":
            legs[str(e)]["one_core_numpy_n1"] = {"env_steps_per_s": _leg(cpus[:1], a.seconds, e, "numpy"),
                                                 "procs": 1}
    first = legs[sorted(legs)[0]]
    src = ("oracle/boat_scalar.py (Python floats + math, f64)" if a.mode == "scalar" else
           "oracle/boat_oracle.py (numpy f64 at N=1)")
    print(json.dumps({
        "config": f"C1: 1 env per process, {src}, per experiment",
        "mode": a.mode,
        "experiments": legs,
        "one_core": first["one_core"], "all_cores": first["all_cores"],
        "os_cpu_count": os.cpu_count(), "affinity_cpus": len(cpus), "cpu_model": _cpu_model(),
        "numpy": np.__version__, "python": platform.python_version(),
        "note": "the reference BoatEnv itself: 13 385 env-steps/s on 1 core, 101 354 on 8 "
                "(SURVEY.md §8(d), survey container)"}))


if __name__ == "__main__":
    main()
