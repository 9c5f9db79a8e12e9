"""The replay path's cost by sampler and exchange (diagnostic, round 6).

bench's workload (exp 6, 65 536 envs); for each configuration bench's own
SegmentRunner + SegmentExchange (as the replay_path field) times N segments:
wall us per step and the median segment launch (HIP events around every launch
on the stepping stream). Configurations: no exchange; the MT-exact draws with the
all-reduce layout (round 5's path); the counter-based draws with the all-reduce
layout; the counter-based draws with the all-gather pack/unpack; the last with the
collective stand-in. Run under `rocprofv3 --kernel-trace --stats` for the
per-kernel durations (k_rb_draw_ctr, k_rb_pack_staged, k_rb_unpack_staged, ...).

    python tools/prof_staged3.py [n_segments]
"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "sac-agent_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    dev = torch.device("cuda", 0)
    base = bench.parse(["--no-cpu-baseline", "--event-every", "1"])
    wl = bench.make_workload(base, 0, dev)
    run0 = bench.SegmentRunner(base, wl, dev)
    run0.prepare()
    k = 0
    for _ in range(24):   # past the clock boost
        k = run0.segment(k, False)
    torch.cuda.synchronize()
    # the staged launch alone (no side work): marks all zero, and a real segment's marks
    # (the philox draws' density, re-copied before each launch: the launch consumes them)
    from sacenv.replay import StagedReplay
    env = wl.envs[0]
    rep = StagedReplay(env.num_envs, env.n_pad, base.experiment, env.first_obs_template(), mem_size=base.replay_mem,
                       batch=base.replay_batch, seg=bench.SEG, device=dev, sampler="philox", exchange="allgather")
    rep.begin(env.obs)
    real = rep.marks[0].clone()
    stage = rep.stage[0]
    marks = torch.zeros_like(real)
    st = torch.cuda.current_stream(dev)
    for name, src in (("plain", None), ("staged-0", "zero"), ("staged-real", real)):
        evs = []
        for _ in range(n):
            if src is not None and name == "staged-real":
                marks.copy_(src)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            if src is None:
                wl.segment_step(k % bench.ACTION_STEPS, bench.SEG)
            else:
                wl.segment_step(k % bench.ACTION_STEPS, bench.SEG, stage=stage, marks=marks)
            b.record(st)
            wl.refill()
            k += bench.SEG
            evs.append((a, b))
        torch.cuda.synchronize()
        ms = [a.elapsed_time(b) * 1e3 for a, b in evs[2:]]
        print(f"launch only {name:12s} median {statistics.median(ms):6.1f} us (min {min(ms):6.1f})", flush=True)
    del rep
    confs = [("none", None, None, False), ("mt", "mt", "allreduce", False), ("philox-ar", "philox", "allreduce", False),
             ("philox-ag", "philox", "allgather", False), ("standin", "philox", "allgather", True)]
    for rnd in range(2):
        for name, smp, xch, sd in confs:
            if smp is None:
                run = bench.SegmentRunner(base, wl, dev)
            else:
                args = bench.parse(["--no-cpu-baseline", "--event-every", "1", "--sampler", smp, "--exchange", xch])
                standin = bench.collective_standin(args, wl) if sd else None
                run = bench.SegmentRunner(args, wl, dev, None, bench.SEG,
                                          bench.make_exchange(args, wl, 0, 1, dev, standin=standin))
            rate, k, _ = bench.timed_rate(run, k, n, 1, dev, wl)
            launches = [a.ms_to(b) * 1e3 for a, b, _ in run.seg_events]
            print(f"r{rnd} {name:10s} {rate['value'] / 1e9:7.3f} G env-steps/s, {rate['ms_per_step'] * 1e3:6.3f} "
                  f"us/step wall, launch median {statistics.median(launches):6.1f} us "
                  f"(min {min(launches):6.1f}, max {max(launches):6.1f})", flush=True)


if __name__ == "__main__":
    main()
