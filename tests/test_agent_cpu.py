"""VecSAC (sacenv.agent) against the reference agent.

``sac_learn.npz`` holds the reference ``ContinuousAgent`` built under
``torch.manual_seed(0)`` and two ``learn()`` calls on fixed batches with
recorded policy noise (tests/golden/make_golden.py::run_sac_learn). On the CPU
the restatement runs the same torch operations, so the losses and every
updated weight agree to float32 rounding.
"""
import numpy as np
import pytest
import torch

from conftest import golden

NETS = ("actor", "critic_1", "critic_2", "value", "target_value")


def run_learn(device, z):
    from sacenv.agent import VecSAC
    cfg = {"agent": {k[4:]: z[k].item() for k in z.files if k.startswith("cfg_")}}
    agent = VecSAC(device, cfg, init_seed=int(z["seed"]), with_memory=False)
    eps = torch.from_numpy(z["eps"])
    losses = []
    for i in range(int(z["n_calls"])):
        b = tuple(torch.from_numpy(z[f"b{i}_{k}"]) for k in ("state", "action", "reward", "new_state", "done"))
        out = agent.learn(b, noise=(eps[2 * i], eps[2 * i + 1]))
        losses.append([float(x) for x in out])
    return agent, np.asarray(losses)


def check(agent, losses, z, rtol_w, rtol_l, init=None):
    mse = z["mse"].reshape(-1, 3)      # per call: value mse, critic 1 mse, critic 2 mse
    np.testing.assert_allclose(losses[:, 0], 0.5 * mse[:, 0], rtol=rtol_l)
    np.testing.assert_allclose(losses[:, 2], 0.5 * mse[:, 1], rtol=rtol_l)
    np.testing.assert_allclose(losses[:, 3], 0.5 * mse[:, 2], rtol=rtol_l)
    for name in NETS:
        for k, v in getattr(agent, name).state_dict().items():
            want = z[f"w_{name}.{k}"]
            got = v.detach().cpu().numpy()
            if init is None:
                err = np.abs(got - want).max()
                assert err <= rtol_w * max(1e-3, np.abs(want).max()), (name, k, err)
            else:
                # across devices: the Adam steps (w - w0), relative to their norm (an
                # entry whose gradient is ~0 may step either way on either device)
                w0 = init[name][k]
                d_ref, d_got = want - w0, got - w0
                n = np.linalg.norm(d_ref)
                if n > 0:
                    assert np.linalg.norm(d_got - d_ref) <= rtol_w * n, (name, k)


def test_vec_sac_learn_matches_reference_cpu():
    z = golden("sac_learn.npz")
    agent, losses = run_learn("cpu", z)
    check(agent, losses, z, rtol_w=1e-6, rtol_l=1e-6)


def test_agent_config_from_reference_yaml():
    from sacenv.agent import AgentConfig
    z = golden("sac_learn.npz")
    c = AgentConfig.from_any({"agent": {k[4:]: z[k].item() for k in z.files if k.startswith("cfg_")}})
    assert c == AgentConfig()  # the defaults are configs/original_config.yaml:12-21


@pytest.mark.gpu
def test_vec_sac_learn_matches_reference_gpu(gpu, built_lib):
    """The same two learn() calls on the MI355X (hipBLASLt GEMMs): fp32 tolerance."""
    z = golden("sac_learn.npz")
    from sacenv.agent import VecSAC
    init = {n: {k: v.numpy().copy() for k, v in sd.items()}
            for n, sd in VecSAC("cpu", init_seed=int(z["seed"]), with_memory=False).state_dicts().items()}
    agent, losses = run_learn(gpu, z)
    check(agent, losses, z, rtol_w=1e-2, rtol_l=1e-4, init=init)
