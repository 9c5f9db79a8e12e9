"""Where the staged launch's extra time comes from (diagnostic, round 6).

bench's workload (exp 6, 65 536 envs), bench's SegmentRunner, the counter-based
draws and the all-gather pack/unpack run serially on the stepping stream (the
replay_path field's schedule). Variants change one thing each and report the wall
rate and the median segment launch (HIP events around every launch):

- none: no exchange (the plain launch);
- ag: the replay path as bench times it (one fused side launch per segment);
- ag-sep: the same with the draws, pack and unpack as three launches;
- ag-zero: the same, the marks zeroed right before each launch (the staged launch
  writes no row; every side kernel still runs);
- ag-plain: the side kernels run, the launch is the plain one (no staged rows);
- evict, evict16, evict256: no exchange, a 96-, 16- or 256-MB fill after each refill
  (does an L2 / MALL sweep between refill and launch slow the launch, and from what
  size?);
- ag-draw-only: the draws run, no pack/unpack;
- rank8: one GPU as rank 0 of the 8-rank buffer (bench's replay_path_rank_of_world);
- rank8-nowait (timing only): the same, the stepping stream not waiting for the
  collective's event before the side launch (its unpack may race the stand-in);
- ag-first, rank8-first: the side launch before the refill instead of after it;
- ag-corun (timing only): the side launch beside the next segment's launch on a side
  stream (the launch does not wait for its draws: marks may race).

    python tools/prof_staged4.py [n_segments] [kind,kind,...]
"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "sac-agent_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
from sacenv.dist import SegmentExchange  # noqa: E402


class Variant(SegmentExchange):
    def __init__(self, sampler, device, kind):
        super().__init__(sampler, device)
        self.kind = kind
        if kind == "ag-sep":   # the draws, pack and unpack as three launches (round 6's first form)
            self.fused = False
        mb = {"evict": 96, "evict16": 16, "evict256": 256}.get(kind)
        self.junk = torch.empty(mb << 20, dtype=torch.uint8, device=device) if mb else None

    def check(self):
        if self.kind != "rank8-nowait":   # (its unpacks may race the stand-in's copies)
            super().check()

    def wait(self):
        if self.kind == "ag-corun":   # the pending unpack reads what the side stream packed
            self._cur().wait_stream(self.sd)
        super().wait()

    def stage_args(self):
        sa = super().stage_args()
        if self.kind == "ag-zero":
            sa["marks"].zero_()
        if self.kind in ("ag-plain", "evict", "evict16", "evict256"):
            return {"stage": None, "marks": None}
        return sa

    def launched(self):
        if self.kind in ("ag-first", "rank8-first"):
            # the side launch right after the segment launch, BEFORE the refill: the refill's
            # fresh slot-ring lines (the next episodes' wind) stay in L2 for the next launch
            g, pend = self.g, self._pending
            if pend is not None and pend[1] is not None:
                self._cur().wait_event(pend[1])
            got = self.sampler.side_segment(g, pend[0] if pend is not None else None)
            if pend is not None:
                self.last = got
            self._pending = (g, None)
            if self.collective:
                packed = self._record(self._cur())
                with torch.cuda.stream(self.coll):
                    self.coll.wait_event(packed)
                    self.sampler.collect_segment(g)
                    self._pending = (g, self._record(self.coll))
            return
        super().launched()

    def after(self):
        if self.kind in ("ag-first", "rank8-first"):
            self.g += 1
            self.exchanges += 1
            return
        if self.kind == "rank8-nowait" and self._pending is not None:
            # TIMING ONLY: the stepping stream does not wait for the collective's event
            self._pending = (self._pending[0], None)
        if self.kind == "ag-corun":
            # TIMING ONLY: the side launch of segment g on a side stream once refill g is
            # done, beside launch g + 1, which does not wait for it (its draws of segment
            # g + 2 then race launch g + 1's marks: rows may be missing)
            ev = self._record(self._cur())
            pend = self._pending
            with torch.cuda.stream(self.sd):
                self.sd.wait_event(ev)
                self.sampler.side_segment(self.g, pend[0] if pend is not None else None)
            self._pending = (self.g, None)
            self.g += 1
            self.exchanges += 1
            return
        if self.kind.startswith("evict"):
            self.junk.fill_(self.g & 0xFF)
            self.g += 1
            self.exchanges += 1
            return
        if self.kind == "ag-draw-only":
            self.sampler.prepare(self.g + 1)
            self.g += 1
            self.exchanges += 1
            return
        super().after()


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    dev = torch.device("cuda", 0)
    base = bench.parse(["--no-cpu-baseline", "--event-every", "1"])
    wl = bench.make_workload(base, 0, dev)
    run0 = bench.SegmentRunner(base, wl, dev)
    run0.prepare()
    k = 0
    for _ in range(24):   # past the clock boost
        k = run0.segment(k, False)
    torch.cuda.synchronize()
    args = bench.parse(["--no-cpu-baseline", "--event-every", "1"])
    kinds = sys.argv[2].split(",") if len(sys.argv) > 2 else ["none", "ag", "ag-sep", "ag-zero", "ag-plain", "evict",
                                                              "ag-draw-only"]
    for rnd in range(2):
        for kind in kinds:
            if kind == "none":
                run = bench.SegmentRunner(base, wl, dev)
            else:
                if kind.startswith("rank8"):   # one GPU as rank 0 of 8, the collective stood in for
                    x = bench.make_exchange(args, wl, 0, 8, dev, standin=bench.collective_standin(args, wl))
                else:
                    x = bench.make_exchange(args, wl, 0, 1, dev)
                v = Variant(x.sampler, dev, kind)
                run = bench.SegmentRunner(args, wl, dev, None, bench.SEG, v)
            rate, k, _ = bench.timed_rate(run, k, n, 1, dev, wl)
            launches = [a.ms_to(b) * 1e3 for a, b, _ in run.seg_events]
            print(f"r{rnd} {kind:13s} {rate['value'] / 1e9:7.3f} G env-steps/s, {rate['ms_per_step'] * 1e3:6.3f} "
                  f"us/step wall, launch median {statistics.median(launches):6.1f} us "
                  f"(min {min(launches):6.1f}, max {max(launches):6.1f})", flush=True)


if __name__ == "__main__":
    main()
