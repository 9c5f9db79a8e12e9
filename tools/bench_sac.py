"""Time the device SAC agent: NativeSAC (sacenv_sac.hip, fp32 MFMA) vs VecSAC (torch).

    python tools/bench_sac.py [--iters 50] [--act-n 65536]

One JSON line: learn() ms per call for both (batch 1024, same batches and
noise; the native call is graph-capturable and timed both eager and as a
hipGraph), choose_action ms for N observations, and the MFMA work per learn
(the dense 256x256 products: 15 per batch row in the row kernels plus the
four fc2 weight gradients) as achieved TFLOP/s against the 157.3 TFLOP/s f32
MFMA peak (MI355X_MICROARCH.md).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sac-agent_amd"))

F32_MFMA_PEAK = 157.3e12


def timed(fn, iters, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--act-n", type=int, default=65536)
    args = ap.parse_args(argv)
    from sacenv.agent import VecSAC
    from sacenv.sac_native import NativeSAC
    dev = torch.device("cuda:0")
    B, H, D = 1024, 256, 11
    g = torch.Generator().manual_seed(0)
    s = (torch.rand((B, D), generator=g)).to(dev)
    a = (torch.rand((B, 1), generator=g) * 2 - 1).to(dev)
    r = torch.rand(B, generator=g, dtype=torch.float64).to(dev)
    s2 = (s + 0.01 * torch.randn((B, D), generator=g).to(dev)).contiguous()
    d = torch.zeros(B, dtype=torch.bool, device=dev)
    e1, e2 = torch.randn((B, 1), device=dev), torch.randn((B, 1), device=dev)
    batch, noise = (s, a, r, s2, d), (e1, e2)
    ref = VecSAC(dev, init_seed=0, with_memory=False)
    nat = NativeSAC(dev, init_seed=0, with_memory=False)
    t_ref = timed(lambda: ref.learn(batch, noise), args.iters)
    t_nat = timed(lambda: nat.learn(batch, noise), args.iters)
    # the four launches of one learn() as a hipGraph (inputs already device f32/f64/u8)
    st, ac = s.contiguous(), a.reshape(-1).contiguous()
    dn = d.to(torch.uint8)
    n1, n2 = e1.reshape(-1).contiguous(), e2.reshape(-1).contiguous()
    nat.learn((st, ac, r, s2, dn), (n1, n2))
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        with torch.cuda.graph(graph, stream=side):
            nat.learn((st, ac, r, s2, dn), (n1, n2))
    torch.cuda.current_stream(dev).wait_stream(side)
    t_graph = timed(graph.replay, args.iters)
    N = args.act_n
    obs = torch.rand((N, D), device=dev)
    eps = torch.randn((N, 1), device=dev)
    t_act_nat = timed(lambda: nat.choose_action(obs, eps=eps), args.iters)
    t_act_ref = timed(lambda: ref.choose_action(obs, eps=eps), args.iters)
    flops_learn = 2.0 * H * H * B * (15 + 4)
    flops_act = 2.0 * H * H * N
    out = {
        "what": "SAC learn() (batch 1024, 256-256 MLPs, f32) and choose_action on one MI355X",
        "learn_ms": {"native_eager": t_nat, "native_graph": t_graph, "torch_vecsac": t_ref},
        "learn_speedup_vs_torch": t_ref / t_graph,
        "choose_action_ms": {"n": N, "native": t_act_nat, "torch_vecsac": t_act_ref},
        "mfma": {"flops_per_learn": flops_learn, "learn_tflops": flops_learn / (t_graph * 1e-3) / 1e12,
                 "act_tflops": flops_act / (t_act_nat * 1e-3) / 1e12, "peak_tflops": F32_MFMA_PEAK / 1e12},
        "iters": args.iters,
    }
    print(json.dumps(out))
    return out


if __name__ == "__main__":
    main()
