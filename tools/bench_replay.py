"""Measurement for the §8(f) replay buffer: one JSON line.

* store: one VecBoatEnv step's transitions (65 536 envs) appended per launch
  pair (k_rb_store + k_rb_advance: store_batch(graph_safe=True), the device-count
  form a captured graph can replay -- each replay appends), graph-replayed; algorithmic bytes per
  transition = read (s 44 + a 4 + r 4 + s' 44 (+ final-obs select) + code 1)
  + write (s 44 + s' 44 + a 4 + r 8 + terminal 1) = 198 B.
* sample: batch 1024 (original_config.yaml:20): the 1 024-thread MT draw + gather.
Timed with HIP events on the launch stream.
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sac-agent_amd"))


def main():
    from sacenv.replay import DeviceReplayBuffer
    dev = torch.device("cuda")
    N, M, B, K = 65536, 1 << 22, 1024, 200
    rb = DeviceReplayBuffer(M, (11,), 1, device=dev, seed=1)
    s = torch.rand(N, 11, device=dev)
    s2 = torch.rand(N, 11, device=dev)
    fin = torch.rand(N, 11, device=dev)
    a = torch.rand(N, 1, device=dev)
    r = torch.rand(N, device=dev)
    code = (torch.rand(N, device=dev) < 0.003).to(torch.uint8)
    for _ in range(3):
        rb.store_batch(s, a, r, s2, code, final_state=fin)
    st = torch.cuda.current_stream()
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(st)
    with torch.cuda.stream(side):
        rb.store_batch(s, a, r, s2, code, final_state=fin, graph_safe=True)
    st.wait_stream(side)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        for _ in range(10):
            rb.store_batch(s, a, r, s2, code, final_state=fin, graph_safe=True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    g.replay()
    torch.cuda.synchronize()
    e0.record(st)
    for _ in range(K // 10):
        g.replay()
    e1.record(st)
    torch.cuda.synchronize()
    store_us = e0.elapsed_time(e1) * 1e3 / K
    rb.mem_cntr = int(rb._cntr.item())
    for _ in range(5):
        rb.sample(B)
    torch.cuda.synchronize()
    e0.record(st)
    for _ in range(K):
        rb.sample(B)
    e1.record(st)
    torch.cuda.synchronize()
    sample_us = e0.elapsed_time(e1) * 1e3 / K
    bytes_store = 198 * N
    print(json.dumps({
        "component": "replay buffer (agent/buffer.py:3-35)",
        "store": {"transitions_per_call": N, "us_per_call": store_us,
                  "transitions_per_s": N / (store_us * 1e-6),
                  "roofline": {"bound": "hbm", "bytes_per_call": bytes_store,
                               "achieved_GBps": bytes_store / (store_us * 1e-6) / 1e9, "peak_GBps": 8000.0,
                               "frac": bytes_store / (store_us * 1e-6) / 8e12}},
        "sample": {"batch": B, "us_per_call_eager": sample_us,
                   "note": "eager launches (draw + gather), host launch overhead included"},
        "capacity": M}))


if __name__ == "__main__":
    main()
