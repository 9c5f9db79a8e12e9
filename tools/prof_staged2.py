"""Which side-stream kernel slows the staged segment launch (diagnostic).

bench's workload (exp 6, 65 536 envs) with a StagedReplay; per segment the launch
is bracketed by HIP events on the stepping stream, and the replay's work is placed:
  serial  -- everything after the refill on the stepping stream (no overlap);
  both    -- draws + marks (prepare) and the gather on the side stream, as bench;
  prep    -- only prepare on the side stream (gather serial after the refill);
  gather  -- only the gather on the side stream (prepare serial);
  after   -- prepare and gather on the side stream after the launch (beside the refill).
Prints the median launch time per mode (us per 256-step launch) and the wall
us per step.
"""
import os
import statistics
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
    env = wl.envs[0]
    from sacenv.replay import StagedReplay
    main_st = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(device=dev)
    for mode in ("plain", "both", "both1", "plain", "both", "both1"):
        rep = StagedReplay(env.num_envs, env.n_pad, args.experiment, env.first_obs_template(), rank=0, world=1,
                           mem_size=args.replay_mem, batch=args.replay_batch, seg=bench.SEG, seed=0, device=dev)
        rep.begin(env.obs)
        k = 0
        launch = []
        ready, done = [], {}
        t_a = t_b = None
        host = []
        for g in range(10):
            h0 = time.perf_counter()
            if g == 3:
                t_a = torch.cuda.Event(enable_timing=True)
                t_a.record(main_st)
            for ev in ready:
                main_st.wait_event(ev)
            ready = []
            if g - 2 in done:   # (implied by ready when prepare follows the gather on the side stream)
                ev = done.pop(g - 2)
                if mode == "both":
                    main_st.wait_event(ev)
            sa = rep.stage_args(g)
            ea, eb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ec = torch.cuda.Event(enable_timing=True)
            ea.record(main_st)
            if mode == "plain":   # no exchange at all (the no-exchange line)
                wl.segment_step(k % bench.ACTION_STEPS, bench.SEG)
            else:
                wl.segment_step(k % bench.ACTION_STEPS, bench.SEG, stage=sa["stage"], marks=sa["marks"])
            eb.record(main_st)
            wl.refill()
            ec.record(main_st)
            k += bench.SEG
            launch.append((ea, eb, ec))
            if mode == "plain":
                host.append(time.perf_counter() - h0)
                continue
            if mode in ("both", "both1", "prep", "after"):
                # as SegmentExchange: prepare(g + 1) does not wait for the launch
                # ("after": it waits for the launch's end, running beside the refill)
                side.wait_event(eb if mode == "after" else ea)
                with torch.cuda.stream(side):
                    rep.prepare(g + 1)
                    e = torch.cuda.Event()
                    e.record(side)
                ready.append(e)
            else:
                rep.prepare(g + 1)
            if mode in ("both", "both1", "gather", "after"):
                side.wait_stream(main_st)
                with torch.cuda.stream(side):
                    rep.sample_segment(g)
                    e = torch.cuda.Event()
                    e.record(side)
                done[g] = e
            else:
                rep.sample_segment(g)
            host.append(time.perf_counter() - h0)
        for ev in ready + list(done.values()):
            main_st.wait_event(ev)
        t_b = torch.cuda.Event(enable_timing=True)
        t_b.record(main_st)
        torch.cuda.synchronize()
        rep.check()
        ms = [a.elapsed_time(b) * 1e3 for a, b, c in launch[3:]]
        rf = statistics.median(b.elapsed_time(c) * 1e3 for a, b, c in launch[3:])
        gap = statistics.median(launch[i][2].elapsed_time(launch[i + 1][0]) * 1e3 for i in range(3, len(launch) - 1))
        per_step = t_a.elapsed_time(t_b) * 1e3 / (7 * bench.SEG)
        print(f"{mode:7s} launch {statistics.median(ms):7.1f} us (min {min(ms):6.1f}), refill {rf:6.1f}, "
              f"refill end -> next launch {gap:6.1f}, host enqueue {statistics.median(host[3:]) * 1e6:6.1f} us; "
              f"{per_step:.3f} us/step "
              f"wall (segments 3-9 with their refills and replay work)", flush=True)


if __name__ == "__main__":
    main()
