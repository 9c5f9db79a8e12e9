"""The staged exchange's side kernels alone, at bench's shape (diagnostic, round 6).

65 536 envs, M = 10^6, B = 1 024, 256-step segments, world 1: each kernel launched
`reps` times back to back between two HIP events (us per launch). The rows the
pack reads are whatever the stage buffers hold (timing only). SACENV_LIB selects a
variant build (tools/variant.py).

    python tools/side_ubench.py [reps]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sac-agent_amd"))

import torch  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    from sacenv import _lib
    from sacenv.replay import StagedReplay
    import ctypes as C
    dev = torch.device("cuda", 0)
    N = 65536
    rep = StagedReplay(N, N, 6, torch.zeros(11), mem_size=1_000_000, batch=1024, seg=256, device=dev,
                       sampler="philox", exchange="allgather")
    rep.begin(torch.zeros(N, 11, device=dev))
    for g in range(2, 6):   # steady-state segments (every learn's range is M)
        rep.prepare(g)
    lib, st = rep.lib, torch.cuda.current_stream(dev)

    def timed(name, fn):
        for _ in range(3):
            fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for _ in range(reps):
            fn()
        b.record(st)
        torch.cuda.synchronize()
        print(f"{name:28s} {a.elapsed_time(b) * 1e3 / reps:8.1f} us", flush=True)

    G = 5
    nb = rep.N_BUFFERS

    def draw(marks=True):
        _lib.check(lib.sacenv_replay_stage_draw_ctr(
            rep._pp, rep._spp, G, rep.batch, rep.seg, 0, rep._idx[G % 4].data_ptr(),
            rep.marks[(G - 1) % nb].data_ptr() if marks else None, rep.marks[G % nb].data_ptr() if marks else None,
            rep._tiles[G % 4].data_ptr(), st.cuda_stream))

    timed("draw (marks, tiles)", draw)
    timed("draw (no marks)", lambda: draw(False))
    timed("pack", lambda: rep.pack_segment(4))
    timed("unpack", lambda: rep.unpack_segment(4))
    rep.drawn = 6

    def side():
        rep.drawn = 6
        rep.side_segment(4, 3)
    timed("side (unpack+pack+draw)", side)
    torch.cuda.synchronize()
    rep.check()


if __name__ == "__main__":
    main()
