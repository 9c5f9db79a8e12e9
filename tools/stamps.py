"""Diagnostic: per-wave phase clocks of k_step from the -DSACENV_STAMPS build.

Builds sac-agent_amd/build/libsacenv_stamps.so (never loaded by the product
path), runs the bench workload for a few hundred steps and prints, per
owner wave: load phase (start -> all loads back), compute phase, store phase,
plus wave start skew and end spread (100 MHz realtime ticks -> us). The accel output region carries the stamps in this
build, so its values are not accelerations.
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "sac-agent_amd")
LIB = os.path.join(PKG, "build", os.environ.get("STAMP_LIB", "libsacenv_stamps.so"))


def build():
    sys.path.insert(0, ROOT)
    import __graft_entry__ as g
    extra = os.environ.get("STAMP_DEFINES", "").split()
    cmd = [g._hipcc(), *g.HIPCC_FLAGS, "-DSACENV_STAMPS", *extra, "-I", os.path.join(ROOT, "include"),
           *[os.path.join(PKG, "csrc", f) for f in g.SOURCES], "-o", LIB]
    subprocess.run(cmd, check=True)


def main():
    if not os.path.exists(LIB) or "--rebuild" in sys.argv:
        build()
    os.environ["SACENV_LIB"] = LIB
    sys.path.insert(0, PKG)
    import numpy as np
    import torch
    from sacenv import VecBoatEnv
    N = int(os.environ.get("STAMP_ENVS", "65536"))
    tm = int(os.environ.get("STAMP_TEST_MODE", "0"))
    env = VecBoatEnv({"base_settings": {"experiment": 6, "test_mode": tm}}, N, device="cuda",
                     max_episode_steps=int(os.environ.get("STAMP_EPISODE", "500")))
    env.reset()
    acts = torch.rand(500, N, device="cuda") * 2 - 1
    nw = env.n_pad // 64
    acc_off = env.layout.accel
    raw = env.arena[acc_off: acc_off + nw * 4 * 8].view(torch.float64).view(nw, 4)
    rows = []
    for k in range(300):  # (VecBoatEnv refills the slot ring by itself every 128 steps)
        env.step_async(acts[k % 500])
        if k >= 100 and k % 10 == 0:
            torch.cuda.synchronize()
            rows.append(raw.cpu().numpy().copy())
    r = np.stack(rows)           # [samples, waves, 4]  realtime start/end, loaded, computed
    t0 = r[..., 0].min(1)
    owner_end = (r[..., 1].max(1) - t0) / 100.0
    print(f"N={N} owner waves={nw} test_mode={tm}")
    print(f"owner span (first owner start -> last owner end) us: median {np.median(owner_end):.2f} "
          f"p90 {np.percentile(owner_end, 90):.2f}")
    for a, b, nm in ((0, 2, "state+wind loads"), (2, 3, "compute"), (3, 1, "stores/end")):
        d = (r[..., b] - r[..., a]) / 100.0
        print(f"    owner {nm:16s} us median {np.median(d):6.2f} p90 {np.percentile(d, 90):6.2f}")
    skew = (r[..., 0] - t0[:, None]) / 100.0
    print(f"owner start skew us: median {np.median(skew):.2f} max {skew.max():.2f}")

if __name__ == "__main__":
    main()
