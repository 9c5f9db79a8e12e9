"""SACENV_SAC_STAMPS diagnostics: per-phase block start/end (us, s_memrealtime 100 MHz) of one learn()."""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sac-agent_amd"))


def main():
    from sacenv.sac_native import NativeSAC
    dev = torch.device("cuda:0")
    B = 1024
    s = torch.rand((B, 11), device=dev)
    a = torch.rand(B, device=dev) * 2 - 1
    r = torch.rand(B, device=dev, dtype=torch.float64)
    d = torch.zeros(B, dtype=torch.uint8, device=dev)
    e = torch.randn(B, device=dev)
    nat = NativeSAC(dev, init_seed=0, with_memory=False)
    res = []
    for it in range(20):
        nat.scratch.zero_()
        nat.learn((s, a, r, s, d), (e, e))
        torch.cuda.synchronize()
        off = (16 * 256 * B + 27 * B + 16 * B)
        st = nat.scratch[off: off + 4 * 1024 * 16 * 2].view(torch.int64).view(4, 1024, 16).cpu()
        res.append(st)
    nblk = {0: 4 * 64, 1: 6 * 64, 2: 4 * 64, 3: 256 + 64 + 1}
    roles = {0: ["actor", "value", "c1stored", "c2stored"], 1: ["c1rs", "c2rs", "c1loss", "c2loss", "c1s", "c2s"],
             2: ["actorbwd0", "actorbwd1", "valuebwd0", "valuebwd1"]}
    for ph in range(4):
        rows = []
        for st in res[5:]:
            t0 = st[ph, :nblk[ph], 0].min().item()
            rows.append((st[ph, :nblk[ph], :] - t0).float() / 100.0)  # us
        med = torch.stack(rows).median(0).values
        if ph < 3:
            for ri, name in enumerate(roles[ph]):
                blk = med[ri * 64:(ri + 1) * 64]
                inner = " ".join(f"p{k} {blk[:, k].median():6.2f}" for k in range(1, 6)) if (ph, ri) == (0, 1) else ""
                print(f"phase {ph} {name:9s} start med {blk[:, 0].median():6.2f} max {blk[:, 0].max():6.2f}  "
                      f"end med {blk[:, 15].median():6.2f} max {blk[:, 15].max():6.2f} {inner}")
        else:
            for name, sl in (("fc2", slice(65, 321)), ("small", slice(1, 65)), ("loss", slice(0, 1))):
                blk = med[sl]
                print(f"phase 3 {name:9s} start med {blk[:, 0].median():6.2f} max {blk[:, 0].max():6.2f}  "
                      f"p1 {blk[:, 1].median():6.2f} p2 {blk[:, 2].median():6.2f} p3 {blk[:, 3].median():6.2f} "
                      f"end med {blk[:, 15].median():6.2f} max {blk[:, 15].max():6.2f}")


if __name__ == "__main__":
    main()
