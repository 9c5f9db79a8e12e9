"""Diagnostic: where the persistent segment kernel's step time goes, by phase.

Builds sac-agent_amd/build/libsacenv_stamps.so with -DSACENV_STAMPS (never
loaded by the product path), runs the bench workload (exp 6, 65 536 envs,
500-step episodes, 128-step segments, no refill between the two measured
segments) and reads the per-wave phase sums the k_rollout owner waves write
into the (otherwise unused) accel region: shader clocks (s_memtime) between
sched-barrier-pinned points of the step (sacenv_boat.hip PHASE):

  1 wind: action, wind piece, trig3 (sin J, sin rudder, sincos wind angle)
  2 dynamics: forces, velocities, yaw, sincos yaw, positions
  3 reward and termination: make_obs, exp reward, penalties, term codes
  4 outputs: counters, restarts, the record (LDS-staged obs block), loop

The barriers themselves cost time (the phases cannot interleave), so the sum
runs above the product kernel's step time; the split is what is read here.
Writes gpurun_out/phase_stamps.json.
"""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "sac-agent_amd")
LIB = os.path.join(PKG, "build", "libsacenv_stamps.so")
NAMES = ("wind", "dynamics", "reward_term", "outputs")


def build():
    sys.path.insert(0, ROOT)
    import __graft_entry__ as g
    cmd = [g._hipcc(), *g.HIPCC_FLAGS, "-DSACENV_STAMPS", "-I", os.path.join(ROOT, "include"),
           *[os.path.join(PKG, "csrc", f) for f in g.SOURCES], "-o", LIB]
    subprocess.run(cmd, check=True)


def main():
    # before anything imports sacenv (build() does, via __graft_entry__): _lib reads
    # SACENV_LIB at import
    os.environ["SACENV_LIB"] = LIB
    if not os.path.exists(LIB) or "--rebuild" in sys.argv or "--build-only" in sys.argv:
        build()
    if "--build-only" in sys.argv:
        return
    os.environ["SACENV_LIB"] = LIB
    sys.path.insert(0, PKG)
    import torch
    from sacenv import VecBoatEnv
    N, K = 65536, 128
    env = VecBoatEnv({"base_settings": {"experiment": 6, "test_mode": 0}}, N, device="cuda",
                     max_episode_steps=500, n_helpers=8192, auto_refill=False)
    env.reset()
    acts = torch.rand(3 * K, N, device="cuda") * 2 - 1
    nw = env.n_pad // 64
    acc = env.arena[env.layout.accel: env.layout.accel + 24 * env.n_pad].view(torch.float64)
    env.segment_async(acts, K)  # warm
    torch.cuda.synchronize()
    out = {"envs": N, "steps_per_launch": K, "segments": []}
    for s in (1, 2):
        acc.zero_()
        ea, eb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ea.record()
        env.segment_async(acts[s * K:], K)
        eb.record()
        torch.cuda.synchronize()
        d = acc[: nw * 8].view(nw, 8).cpu().numpy()
        if not (d[:, 4] == K).all():
            raw = acc[: 64].cpu().numpy()
            raise SystemExit(f"phase stamps missing: counts {np.unique(d[:, 4])[:8]}, first doubles {raw[:16]}, "
                             f"lib {os.environ.get('SACENV_LIB')}")
        per_step = d[:, :4] / K
        med = np.median(per_step, axis=0)
        total = float(med.sum())
        us = ea.elapsed_time(eb) * 1e3 / K
        seg = {"us_per_step": us, "cycles_per_step": total, "ghz_implied": total / (us * 1e3),
               "phases_cycles": {n: float(v) for n, v in zip(NAMES, med)},
               "phases_frac": {n: float(v / total) for n, v in zip(NAMES, med)},
               "p90_cycles": {n: float(v) for n, v in zip(NAMES, np.percentile(per_step, 90, axis=0))}}
        out["segments"].append(seg)
        print(json.dumps(seg))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "phase_stamps.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
