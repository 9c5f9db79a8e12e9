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
    for g in range(6):     # serialised: one stream
        wl.segment_step(k % bench.ACTION_STEPS, bench.SEG, trans=rep.rows(g))
        wl.refill()
        rep.sample_segment(g)
        k += bench.SEG
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for g in range(6, 12):
        wl.segment_step(k % bench.ACTION_STEPS, bench.SEG, trans=rep.rows(g))
        wl.refill()
        rep.sample_segment(g)
        k += bench.SEG
    torch.cuda.synchronize()
    ser = (time.perf_counter() - t0) / (6 * bench.SEG)
    run = bench.SegmentRunner(args, wl, dev, None, bench.SEG, x)
    x.g = 12
    x.started = True
    rate, k, _ = bench.timed_rate(run, k, 6, 1, dev, wl)
    print(f"serialised {ser * 1e6:.3f} us/step; overlapped {rate['ms_per_step'] * 1e3:.3f} us/step "
          f"({rate['value'] / 1e9:.2f} G env-steps/s)", flush=True)


if __name__ == "__main__":
    main()
