"""Profile the staged replay path (rocprofv3 --kernel-trace --stats target).

bench's workload (exp 6, 65 536 envs), persistent segments writing their
transition rows into a StagedReplay, each segment's 256 learns sampled after
it on the same stream (serialised, so the kernel trace shows each kernel's own
duration), then the same with the exchange on its side stream (overlapped).
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "sac-agent_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    args = bench.parse(["--no-cpu-baseline"])
    dev = torch.device("cuda", 0)
    wl = bench.make_workload(args, 0, dev)
    x = bench.make_exchange(args, wl, 0, 1, dev)
    rep, env = x.sampler, wl.envs[0]
    rep.begin(env.obs)
    k = 0

    def seg(g):
        nonlocal k
        sa = rep.stage_args(g)
        wl.segment_step(k % bench.ACTION_STEPS, bench.SEG, stage=sa["stage"], marks=sa["marks"])
        wl.refill()
        rep.prepare(g + 1)
        rep.sample_segment(g)
        k += bench.SEG

    for g in range(6):     # serialised: one stream
        seg(g)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for g in range(6, 12):
        seg(g)
    torch.cuda.synchronize()
    ser = (time.perf_counter() - t0) / (6 * bench.SEG)
    # the no-exchange segment for reference
    t0 = time.perf_counter()
    for g in range(6):
        wl.segment_step(k % bench.ACTION_STEPS, bench.SEG)
        wl.refill()
        k += bench.SEG
    torch.cuda.synchronize()
    plain = (time.perf_counter() - t0) / (6 * bench.SEG)
    x = bench.make_exchange(args, wl, 0, 1, dev)
    run = bench.SegmentRunner(args, wl, dev, None, bench.SEG, x)
    rate, k, _ = bench.timed_rate(run, k, 6, 1, dev, wl)
    print(f"no exchange {plain * 1e6:.3f} us/step; serialised {ser * 1e6:.3f} us/step; overlapped "
          f"{rate['ms_per_step'] * 1e3:.3f} us/step ({rate['value'] / 1e9:.2f} G env-steps/s)", flush=True)


if __name__ == "__main__":
    main()
