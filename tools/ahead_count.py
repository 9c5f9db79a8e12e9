"""Diagnostic: how many envs the refill's twist-ahead serves (bench workload).

Per 256-step segment of exp 6 at 65 536 envs: envs whose MT position wrapped
(their draws crossed into the pre-twisted block, which the fit launch then made
current and twisted the next one), and envs left without the pre-twisted block
after the refill (should be none).
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
        p0 = env.mt_pos.clone()
        wl.segment_step(k % bench.ACTION_STEPS, bench.SEG)
        wl.refill()
        k += bench.SEG
        torch.cuda.synchronize()
        p1 = env.mt_pos
        pos0, pos1 = p0 & 0xFFFF, p1 & 0xFFFF
        print(f"segment {g}: wrapped {int((pos1 < pos0).sum())}, moved {int((pos1 != pos0).sum())}, "
              f"without next block {int(((p1 >> 16) & 1 == 0).sum())}, pos max {int(pos1.max())}", flush=True)


if __name__ == "__main__":
    main()
