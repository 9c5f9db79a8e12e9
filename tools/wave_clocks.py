"""Diagnostic: how the persistent segment's launch time splits into wave lives.

Builds libsacenv_wclk.so (tools/variant.py: each k_rollout owner wave stores
its s_memrealtime at entry and after its last store is issued, its XCC id and
HW_ID into the accel region; never loaded by the product path), runs bench's
workload (exp 6, 65 536 envs, 256-step segments with their refills) and, for
a few segments, reports the spread of wave starts and ends, the mean and
maximum wave life per step, and per-XCD / per-SIMD-slot means, next to the
launch duration from HIP events. Writes gpurun_out/wave_clocks.json.

    python tools/wave_clocks.py build      (here, on the CPU)
    python tools/wave_clocks.py            (on the GPU box)
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "sac-agent_amd", "build", "libsacenv_wclk.so")

START = ("#ifdef SACENV_STAMPS\n  const uint64_t st_real0 = __builtin_amdgcn_s_memrealtime();",
         "const uint64_t wclk0 = __builtin_amdgcn_s_memrealtime();\n"
         "#ifdef SACENV_STAMPS\n  const uint64_t st_real0 = __builtin_amdgcn_s_memrealtime();")
END = ("#ifdef SACENV_STAMPS\n  asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");\n  if (kRoll && lane == 0) {",
       "if (kRoll && lane == 0) {\n"
       "    uint32_t wx, wh;\n"
       "    asm volatile(\"s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)\" : \"=s\"(wx));\n"
       "    asm volatile(\"s_getreg_b32 %0, hwreg(HW_REG_HW_ID)\" : \"=s\"(wh));\n"
       "    double* wd = A.accel() + (int64_t)ob * 4;\n"
       "    wd[0] = (double)wclk0; wd[1] = (double)__builtin_amdgcn_s_memrealtime();\n"
       "    wd[2] = (double)wx; wd[3] = (double)wh;\n"
       "  }\n"
       "#ifdef SACENV_STAMPS\n  asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");\n  if (kRoll && lane == 0) {")


def build():
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "variant.py"), "wclk", *START, *END],
                   check=True)


def main():
    os.environ["SACENV_LIB"] = LIB
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "sac-agent_amd"))
    import numpy as np
    import torch
    import bench
    args = bench.parse(["--no-cpu-baseline"])
    dev = torch.device("cuda", 0)
    wl = bench.make_workload(args, 0, dev)
    env = wl.envs[0]
    nw = env.n_pad // 64
    k = 0
    out = []
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for g in range(64):   # (the clock boosts after ~20 launches: report the steady state)
        e0.record()
        wl.segment_step(k % bench.ACTION_STEPS, bench.SEG)
        e1.record()
        wl.refill()
        k += bench.SEG
        if g < 56:   # back to back, as the bench runs them (the clock boosts after ~20 launches)
            continue
        torch.cuda.synchronize()
        d = env.accel.reshape(-1)[: 4 * nw].view(nw, 4).cpu().numpy()
        t0, t1 = d[:, 0], d[:, 1]
        life = (t1 - t0) / 100.0 / bench.SEG      # s_memrealtime: 100 MHz
        xcc = d[:, 2].astype(np.int64)
        hw = d[:, 3].astype(np.int64)
        simd = (hw >> 4) & 3
        cu = (hw >> 8) & 15
        se = (hw >> 13) & 7
        rec = {
            "event_us_per_step": e0.elapsed_time(e1) * 1e3 / bench.SEG,
            "span_us_per_step": (t1.max() - t0.min()) / 100.0 / bench.SEG,
            "start_spread_us": (t0.max() - t0.min()) / 100.0,
            "end_spread_us": (t1.max() - t1.min()) / 100.0,
            "life_us_per_step": {"mean": float(life.mean()), "min": float(life.min()),
                                 "p50": float(np.median(life)), "p90": float(np.percentile(life, 90)),
                                 "max": float(life.max())},
            "per_xcc_mean": [float(life[xcc == x].mean()) for x in range(8) if (xcc == x).any()],
            "per_xcc_max": [float(life[xcc == x].max()) for x in range(8) if (xcc == x).any()],
            "per_simd_mean": [float(life[simd == s].mean()) for s in range(4)],
            "waves_per_cu_max": int(np.bincount(xcc * 512 + se * 64 + cu * 4 + simd).max()),
        }
        if g == 63:
            order = np.argsort(life)
            rec["slowest"] = [{"wave": int(i), "life": float(life[i]), "xcc": int(xcc[i]), "se": int(se[i]),
                               "cu": int(cu[i]), "simd": int(simd[i])} for i in order[-8:]]
            rec["hist"] = np.histogram(life, bins=12)[0].tolist()
            rec["hist_edges"] = [round(float(x), 4) for x in np.histogram(life, bins=12)[1]]
        out.append(rec)
        print(json.dumps({k2: v for k2, v in rec.items() if k2 not in ("slowest", "hist", "hist_edges")}),
              flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(out, open(os.path.join(ROOT, "gpurun_out", "wave_clocks.json"), "w"), indent=1)
    print(json.dumps(out[-1].get("slowest")), out[-1].get("hist"), out[-1].get("hist_edges"))


if __name__ == "__main__":
    build() if sys.argv[1:] == ["build"] else main()
