"""Diagnostic: how the episodes a refill draws spread over the envs (bench workload).

Per 256-step segment of exp 6 at 65 536 envs: episodes started per env (the
difference of the arena's `cons` around the segment), as a histogram, with the
mean over the envs that started any and the maximum -- k_refill's 16-lane group
draws one env's episodes one after the other, so the busiest env bounds it.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "sac-agent_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    args = bench.parse(["--no-cpu-baseline"])
    dev = torch.device("cuda", 0)
    wl = bench.make_workload(args, 0, dev)
    env = wl.envs[0]
    k = 0
    for g in range(12):
        c0 = env.cons.clone()
        wl.segment_step(k % bench.ACTION_STEPS, bench.SEG)
        wl.refill()
        k += bench.SEG
        torch.cuda.synchronize()
        d = (env.cons - c0).cpu()
        if g < 4:
            continue
        nz = d[d > 0]
        hist = torch.bincount(d.clamp(max=20)).tolist()
        print(f"segment {g}: envs with episodes {nz.numel()}, episodes {int(d.sum())}, mean over those "
              f"{nz.float().mean():.2f}, max {int(d.max())}, histogram (0..20+) {hist}", flush=True)


if __name__ == "__main__":
    main()
