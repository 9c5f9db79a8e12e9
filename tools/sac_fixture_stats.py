"""Per-tensor agreement of the GPU agents with the reference learn() fixture
(tests/golden/sac_learn.npz): for each weight tensor, the Adam steps (w - w0) of
NativeSAC (MFMA kernels) and VecSAC (torch on the GPU) against the reference's.

Adam's first steps are ~lr * sign(g) per entry (m / sqrt(v) with one or two
gradients), so an entry whose gradient is within fp32 accumulation error of 0 can
step the other way on another device: such "flips" differ by ~2 lr whatever the
kernel. Reported per tensor: entries, flips (|d - d_ref| > 0.5 |d_ref|), the step
error relative to the step norm with and without the flips.

    python tools/sac_fixture_stats.py > gpurun_out/sac_fixture_stats.json
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sac-agent_amd"), os.path.join(ROOT, "tests")]

from conftest import golden  # noqa: E402

NETS = ("actor", "critic_1", "critic_2", "value", "target_value")


def run(kind, z, dev):
    from sacenv.agent import VecSAC
    from sacenv.sac_native import NativeSAC
    cfg = {"agent": {k[4:]: z[k].item() for k in z if k.startswith("cfg_")}}
    if kind == "native":
        agent = NativeSAC(dev, cfg, init_seed=int(z["seed"]), with_memory=False)
    else:
        agent = VecSAC(dev, cfg, init_seed=int(z["seed"]), with_memory=False)
    eps = torch.from_numpy(z["eps"])
    for i in range(int(z["n_calls"])):
        b = tuple(torch.from_numpy(z[f"b{i}_{k}"]).to(dev) for k in ("state", "action", "reward", "new_state",
                                                                      "done"))
        agent.learn(b, noise=(eps[2 * i].to(dev), eps[2 * i + 1].to(dev)))
    torch.cuda.synchronize()
    return agent


def main():
    from sacenv.agent import VecSAC
    z = golden("sac_learn.npz")
    dev = torch.device("cuda", 0)
    init = {n: {k: v.numpy().copy() for k, v in sd.items()}
            for n, sd in VecSAC("cpu", init_seed=int(z["seed"]), with_memory=False).state_dicts().items()}
    out = {}
    for kind in ("native", "torch_gpu"):
        agent = run(kind, z, dev)
        rows = {}
        for n in NETS:
            for k, v in getattr(agent, n).state_dict().items():
                want = z[f"w_{n}.{k}"].astype(np.float64)
                got = v.detach().cpu().numpy().astype(np.float64)
                w0 = init[n][k].astype(np.float64)
                d_ref, d = want - w0, got - w0
                nrm = float(np.linalg.norm(d_ref))
                if nrm == 0:
                    continue
                flip = np.abs(d - d_ref) > 0.5 * np.abs(d_ref)
                keep = ~flip
                rows[f"{n}.{k}"] = {
                    "entries": int(d.size), "flips": int(flip.sum()),
                    "rel_err": float(np.linalg.norm(d - d_ref) / nrm),
                    "rel_err_no_flips": float(np.linalg.norm((d - d_ref)[keep]) / max(np.linalg.norm(d_ref[keep]), 1e-300)),
                    "max_entry_err_no_flips_over_step": float(np.max(np.abs(d - d_ref)[keep] / np.maximum(np.abs(d_ref[keep]), 1e-30)))
                    if keep.any() else 0.0,
                }
        out[kind] = rows
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
