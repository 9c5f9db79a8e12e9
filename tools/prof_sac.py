"""Native SAC kernels only (for rocprofv3 traces): N learn() calls and N choose_action calls."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sac-agent_amd"))


def main(n=50):
    from sacenv.sac_native import NativeSAC
    dev = torch.device("cuda:0")
    B = 1024
    s = torch.rand((B, 11), device=dev)
    a = torch.rand(B, device=dev) * 2 - 1
    r = torch.rand(B, device=dev, dtype=torch.float64)
    d = torch.zeros(B, dtype=torch.uint8, device=dev)
    e = torch.randn(B, device=dev)
    nat = NativeSAC(dev, init_seed=0, with_memory=False)
    obs = torch.rand((65536, 11), device=dev)
    eo = torch.randn(65536, device=dev)
    for _ in range(n):
        nat.learn((s, a, r, s, d), (e, e))
    for _ in range(n):
        nat.choose_action(obs, eps=eo)
    torch.cuda.synchronize()
    print("done", [float(x) for x in nat.losses.cpu()])


if __name__ == "__main__":
    main()
