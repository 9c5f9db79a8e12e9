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
    cfg = {"agent": {k[4:]: z[k].item() for k in z if k.startswith("cfg_")}}
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
    # the losses the reference's three backward() calls start from (value, actor,
    # critic_1 + critic_2; continuous_agent.py:123,138,150): the actor loss too
    bwd = z["backward_losses"].reshape(-1, 3)
    np.testing.assert_allclose(losses[:, 0], bwd[:, 0], rtol=rtol_l)
    np.testing.assert_allclose(losses[:, 1], bwd[:, 1], rtol=rtol_l)
    np.testing.assert_allclose(losses[:, 2] + losses[:, 3], bwd[:, 2], rtol=rtol_l)
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
    c = AgentConfig.from_any({"agent": {k[4:]: z[k].item() for k in z if k.startswith("cfg_")}})
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


def _fixture_batches(z, device="cpu"):
    eps = torch.from_numpy(z["eps"])
    for i in range(int(z["n_calls"])):
        b = tuple(torch.from_numpy(z[f"b{i}_{k}"]).to(device)
                  for k in ("state", "action", "reward", "new_state", "done"))
        yield b, (eps[2 * i].to(device), eps[2 * i + 1].to(device))


def checkpoint_round_trip(make, device, tmp_path, optimizer):
    """ContinuousAgent.save_models / load_models (continuous_agent.py:79-91,
    networks/base_network.py:13-17): agent A learns, saves; a fresh agent B with
    other initial weights loads; then both learn the same batch -> bit-identical
    losses and weights. Without the optimizer file B's Adam starts fresh, so A is
    saved before its first learn(); with it, after two."""
    from sacenv.agent import CHECKPOINT_NAMES
    z = golden("sac_learn.npz")
    batches = list(_fixture_batches(z, device))
    a, b = make(0), make(5)
    if optimizer:
        for bt, nz in batches:
            a.learn(bt, noise=nz)
    a.save_models(str(tmp_path), optimizer=optimizer)
    # the reference's files: one plain state_dict per net, under its network name
    for n, fname in CHECKPOINT_NAMES.items():
        sd = torch.load(tmp_path / "checkpoints" / fname, weights_only=True)
        assert list(sd) == list(getattr(a, n).state_dict()), n
    b.load_models(str(tmp_path), optimizer=optimizer)
    bt, nz = batches[1]
    la, lb = a.learn(bt, noise=nz), b.learn(bt, noise=nz)
    assert [float(x) for x in la] == [float(x) for x in lb]
    for n in NETS:
        for k, v in getattr(a, n).state_dict().items():
            assert torch.equal(v, getattr(b, n).state_dict()[k]), (n, k)


@pytest.mark.parametrize("optimizer", [False, True])
def test_vec_sac_checkpoint_round_trip_cpu(tmp_path, optimizer):
    from sacenv.agent import VecSAC
    checkpoint_round_trip(lambda s: VecSAC("cpu", init_seed=s, with_memory=False), "cpu", tmp_path,
                          optimizer)
