"""Diagnostic: where k_refill's time goes, from non-serialising phase clocks.

Builds sac-agent_amd/build/libsacenv_stamps.so with -DSACENV_STAMPS (never loaded by
the product path), runs the bench workload (exp 6, 65 536 envs, 500-step episodes,
persistent 128-step segments) and after each of a few refills reads the per-wave
clocks k_refill writes into the (otherwise unused) accel region and k_refill_fit's
per-block start/end in the reward64 region. A clock is taken once the values it
names are in registers; no other wait is inserted (sacenv_boat.hip REFILL_STAMP).

Per refill wave (round 3, grouped draw): start, status read, the four-env fast path
done, the end of each wave-per-env draw that follows (the first 19), end, draw count.
Prints medians / percentiles in us (100 MHz s_memrealtime) and writes the summary
as JSON to gpurun_out/refill_stamps.json.
"""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "sac-agent_amd")
LIB = os.path.join(PKG, "build", "libsacenv_stamps.so")


def build():
    sys.path.insert(0, ROOT)
    import __graft_entry__ as g
    cmd = [g._hipcc(), *g.HIPCC_FLAGS, "-DSACENV_STAMPS", "-I", os.path.join(ROOT, "include"),
           *[os.path.join(PKG, "csrc", f) for f in g.SOURCES], "-o", LIB]
    subprocess.run(cmd, check=True)


def pct(x):
    x = np.asarray(x, np.float64)
    if x.size == 0:
        return None
    return {"median": float(np.median(x)), "p10": float(np.percentile(x, 10)),
            "p90": float(np.percentile(x, 90)), "max": float(x.max()), "n": int(x.size)}


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
    N, H = 65536, 8192
    env = VecBoatEnv({"base_settings": {"experiment": 6, "test_mode": 0}}, N, device="cuda",
                     max_episode_steps=500, n_helpers=H, auto_refill=False)
    env.reset()
    acts = torch.rand(512, N, device="cuda") * 2 - 1
    acc = env.arena[env.layout.accel: env.layout.accel + 24 * env.n_pad].view(torch.int64).view(-1, 24)
    fit = env.arena[env.layout.reward64: env.layout.reward64 + 8 * env.n_pad].view(torch.int64).view(-1, 2)
    samples = []
    for s in range(12):
        env.segment_async(acts[(128 * s) % 512:], 128)
        torch.cuda.synchronize()
        acc.zero_()
        fit.zero_()
        env.refill()
        torch.cuda.synchronize()
        if s >= 4:  # past the start-up transient
            samples.append((acc[:H].cpu().numpy().copy(), fit[:H].cpu().numpy().copy(),
                            int(env.status[2].item())))
    tick = 0.01  # us per 100 MHz tick
    out = {"envs": N, "helpers": H, "refills": []}
    agg = {k: [] for k in ("read_total", "fast_path", "wave_draw", "slow_tail", "wave_span", "start_skew",
                           "end_spread", "wave_draws", "fit_start", "fit_block", "fit_end", "fit_exit_start",
                           "refill_to_fit_gap")}
    for a, f, ranked in samples:
        live = a[:, 0] > 0
        a = a[live].astype(np.float64)
        t0 = a[:, 0].min()
        agg["start_skew"] += list((a[:, 0] - t0) * tick)
        agg["end_spread"] += list((a[:, 22] - t0) * tick)
        agg["wave_span"] += list((a[:, 22] - a[:, 0]) * tick)
        agg["read_total"] += list((a[:, 1] - a[:, 0]) * tick)
        agg["fast_path"] += list((a[:, 2] - a[:, 1]) * tick)
        n_dr = a[:, 23].astype(int)
        agg["wave_draws"] += list(n_dr)
        for r, n in zip(a, n_dr):
            prev = r[2]
            for j in range(min(n, 19)):
                agg["wave_draw"].append((r[3 + j] - prev) * tick)
                prev = r[3 + j]
            if n:
                agg["slow_tail"].append((r[22] - r[2]) * tick)
        fl = f[f[:, 0] > 0].astype(np.float64)
        fit_span = (fl[:, 1].max() - fl[:, 0].min()) * tick if (fl[:, 1] > 0).any() else None
        if fit_span is not None:  # blocks that fitted (end stamp): start skew, duration
            fw = fl[fl[:, 1] > 0]
            f0 = fl[:, 0].min()
            agg["fit_start"] += list((fw[:, 0] - f0) * tick)
            agg["fit_block"] += list((fw[:, 1] - fw[:, 0]) * tick)
            agg["fit_end"] += list((fw[:, 1] - f0) * tick)
            agg["fit_exit_start"] += list((fl[fl[:, 1] == 0][:, 0] - f0) * tick)
            agg["refill_to_fit_gap"] += [float((f0 - a[:, 22].max()) * tick)]
        out["refills"].append({"listed_envs": ranked, "k_refill_span_us": float((a[:, 22].max() - t0) * tick),
                               "waves_with_wave_draws": int((n_dr > 0).sum()), "k_refill_fit_span_us": fit_span})
    out["phases_us"] = {k: pct(v) for k, v in agg.items()}
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "refill_stamps.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    for r in out["refills"]:
        print("refill:", r)
    for k, v in out["phases_us"].items():
        print(f"{k:12s}", v and {kk: round(vv, 3) for kk, vv in v.items()})


if __name__ == "__main__":
    main()
