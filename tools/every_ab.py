"""The every-output rollout (bench.py's every_output field) and the in-place segment line,
alternating, for A/B builds (SACENV_LIB; diagnostic, round 6).

    python tools/every_ab.py [n_segments]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "sac-agent_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    dev = torch.device("cuda", 0)
    args = bench.parse(["--no-cpu-baseline", "--event-every", "1"])
    wl = bench.make_workload(args, 0, dev)
    run = bench.SegmentRunner(args, wl, dev)
    run.prepare()
    k = 0
    for _ in range(24):   # past the clock boost
        k = run.segment(k, False)
    torch.cuda.synchronize()
    for rnd in range(3):
        e = bench.every_output_rate(wl, dev, n_segs=n, k0=k)
        k += (n + 2) * bench.SEG
        rate, k, _ = bench.timed_rate(run, k, n, 1, dev, wl)
        print(f"r{rnd} every_output {e['value'] / 1e9:7.3f} G ({e['ms_per_step'] * 1e3:6.3f} us/step), "
              f"segments {rate['value'] / 1e9:7.3f} G ({rate['ms_per_step'] * 1e3:6.3f} us/step)", flush=True)


if __name__ == "__main__":
    main()
