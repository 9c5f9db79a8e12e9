"""NativeSAC (sacenv_sac.hip) against the torch fp32 agent.

The floating-point reference for the MFMA kernels is VecSAC (sacenv/agent.py):
the torch restatement of ContinuousAgent that tests/test_agent_cpu.py pins to
the reference agent itself (``sac_learn.npz``). Both are f32; only summation
orders differ, so the tolerances are f32 ones:

* choose_action: actions and log-probs within 2e-5 (absolute, values O(1));
* gradients: with Adam's eps set to 1e3 an Adam step is -lr * g / 1e3 to
  within |g| / 1e3, i.e. linear in the gradient, so the parameter change of
  one learn() compares the gradients of all four losses: per tensor within
  1e-3 of the change's norm;
* losses within 1e-4 relative; the target soft update bit-exact (the same
  f32 ops in the same order);
* the reference fixture: the two recorded learn() calls, Adam steps within
  1e-2 of their norm (the GPU VecSAC test's bar: an entry whose gradient is ~0
  may step either way).
"""
import numpy as np
import pytest
import torch

from conftest import golden

NETS = ("actor", "critic_1", "critic_2", "value", "target_value")
pytestmark = pytest.mark.gpu


def _pair(gpu, seed=0, adam_eps=1e-8, cfg=None):
    from sacenv.agent import VecSAC
    from sacenv.sac_native import NativeSAC
    ref = VecSAC(gpu, cfg, init_seed=seed, with_memory=False)
    nat = NativeSAC(gpu, cfg, init_seed=seed, with_memory=False, adam_eps=adam_eps)
    if adam_eps != 1e-8:
        for opt in (ref.opt_actor, ref.opt_c1, ref.opt_c2, ref.opt_value):
            for g in opt.param_groups:
                g["eps"] = adam_eps
    return ref, nat


def _batch(gpu, B=1024, seed=1):
    g = torch.Generator().manual_seed(seed)
    s = torch.rand((B, 11), generator=g) * 1.2 - 0.1
    a = torch.rand((B, 1), generator=g) * 2 - 1
    r = (torch.rand(B, generator=g, dtype=torch.float64) - 0.8) * 3
    s2 = s + 0.01 * torch.randn((B, 11), generator=g)
    d = torch.rand(B, generator=g) < 0.1
    e1, e2 = torch.randn((B, 1), generator=g), torch.randn((B, 1), generator=g)
    dev = lambda x: x.to(gpu)  # noqa: E731
    return tuple(map(dev, (s, a, r, s2, d))), (dev(e1), dev(e2))


def _weights(agent):
    return {n: {k: v.detach().float().cpu().numpy().copy() for k, v in sd.items()}
            for n, sd in agent.state_dicts().items()}


def test_native_weights_are_the_reference_init(gpu, built_lib):
    ref, nat = _pair(gpu, seed=3)
    a, b = _weights(ref), _weights(nat)
    for n in NETS:
        for k in a[n]:
            np.testing.assert_array_equal(a[n][k], b[n][k], err_msg=f"{n}.{k}")


@pytest.mark.parametrize("n", [1, 37, 1000, 65536])
def test_native_choose_action_matches_torch(gpu, built_lib, n):
    ref, nat = _pair(gpu, seed=5)
    g = torch.Generator().manual_seed(n)
    obs = (torch.rand((n, 11), generator=g) * 1.2 - 0.1).to(gpu)
    eps = torch.randn((n, 1), generator=g).to(gpu)
    got = nat.choose_action(obs, eps=eps)
    with torch.no_grad():
        want, _ = ref.actor.sample_normal(obs, reparameterize=False, eps=eps)
    torch.cuda.synchronize()
    assert got.shape == (n, 1)
    np.testing.assert_allclose(got.cpu().numpy(), want.cpu().numpy(), atol=2e-5, rtol=0)


def test_native_learn_gradients_match_torch(gpu, built_lib):
    """One learn() with Adam in its linear regime: every parameter's change ~ its gradient."""
    ref, nat = _pair(gpu, seed=0, adam_eps=1e3)
    w0 = _weights(ref)
    batch, noise = _batch(gpu)
    lr = ref.learn(batch, noise)
    ln = nat.learn(batch, noise)
    torch.cuda.synchronize()
    np.testing.assert_allclose([float(x) for x in ln], [float(x) for x in lr], rtol=1e-4)
    a, b = _weights(ref), _weights(nat)
    for n in NETS:
        for k in a[n]:
            d_ref, d_nat = a[n][k] - w0[n][k], b[n][k] - w0[n][k]
            nrm = np.linalg.norm(d_ref)
            err = np.linalg.norm(d_nat - d_ref)
            if n == "target_value":  # tau * a step that is already ~lr * g / 1e3: below f32 resolution in places
                assert err <= 1e-3 * nrm + 1e-9, (n, k, err, nrm)
                continue
            assert nrm > 0, (n, k)
            assert err <= 1e-3 * nrm, (n, k, err / nrm)


def test_native_target_soft_update_is_exact(gpu, built_lib):
    ref, nat = _pair(gpu, seed=2)
    t0 = {k: v.clone() for k, v in nat.target_value.state_dict().items()}
    batch, noise = _batch(gpu, seed=4)
    nat.learn(batch, noise)
    tau = nat.cfg.tau
    for k, v in nat.value.state_dict().items():
        want = tau * v + (1 - tau) * t0[k]
        assert torch.equal(nat.target_value.state_dict()[k], want), k


def test_native_learn_matches_reference_fixture(gpu, built_lib):
    """The two reference learn() calls of sac_learn.npz (as test_agent_cpu.py)."""
    from sacenv.agent import VecSAC
    from sacenv.sac_native import NativeSAC
    from test_agent_cpu import check
    z = golden("sac_learn.npz")
    cfg = {"agent": {k[4:]: z[k].item() for k in z if k.startswith("cfg_")}}
    init = {n: {k: v.numpy().copy() for k, v in sd.items()}
            for n, sd in VecSAC("cpu", init_seed=int(z["seed"]), with_memory=False).state_dicts().items()}
    agent = NativeSAC(gpu, cfg, init_seed=int(z["seed"]), with_memory=False)
    eps = torch.from_numpy(z["eps"])
    losses = []
    for i in range(int(z["n_calls"])):
        b = tuple(torch.from_numpy(z[f"b{i}_{k}"]) for k in ("state", "action", "reward", "new_state", "done"))
        out = agent.learn(b, noise=(eps[2 * i], eps[2 * i + 1]))
        losses.append([float(x) for x in out])
    # bar: every weight tensor's two Adam steps within 1e-3 of their
    # norm; measured worst 6.8e-5 (actor.fc2.weight; tools/sac_fixture_stats.py,
    # profiles/r04_sac_fixture_stats.json: no entry steps the other way)
    check(agent, np.asarray(losses), z, rtol_w=1e-3, rtol_l=1e-4, init=init)


def test_native_learn_tracks_torch_over_steps(gpu, built_lib):
    """Ten learn() calls on fresh batches: the two agents stay together (Adam at its defaults)."""
    ref, nat = _pair(gpu, seed=7)
    w0 = _weights(ref)
    for i in range(10):
        batch, noise = _batch(gpu, seed=100 + i)
        lr = ref.learn(batch, noise)
        ln = nat.learn(batch, noise)
    torch.cuda.synchronize()
    np.testing.assert_allclose([float(x) for x in ln], [float(x) for x in lr], rtol=2e-3, atol=1e-6)
    a, b = _weights(ref), _weights(nat)
    for n in NETS:
        for k in a[n]:
            d_ref, d_nat = a[n][k] - w0[n][k], b[n][k] - w0[n][k]
            nrm = np.linalg.norm(d_ref)
            # (was 2e-2) measured worst 2.0e-4, value.fc2.weight
            assert np.linalg.norm(d_nat - d_ref) <= 2e-3 * nrm + 1e-7, (n, k)


def test_native_learn_from_device_buffer(gpu, built_lib):
    """learn() with no batch samples the device replay buffer (buffer.py:24-35)."""
    from sacenv.sac_native import NativeSAC
    nat = NativeSAC(gpu, init_seed=0, with_memory=True)
    assert nat.learn() is None  # mem_cntr < batch_size (:97-98)
    n = 2048
    g = torch.Generator().manual_seed(9)
    s = torch.rand((n, 11), generator=g).to(gpu)
    a = torch.rand((n, 1), generator=g).to(gpu) * 2 - 1
    r = torch.rand(n, generator=g, dtype=torch.float64).to(gpu)
    code = torch.zeros(n, dtype=torch.uint8, device=gpu)
    nat.memory.store_batch(s, a, r, s, code)
    out = nat.learn()
    torch.cuda.synchronize()
    assert out is not None and all(np.isfinite(float(x)) for x in out)


def test_native_rejects_bad_shapes(gpu, built_lib):
    from sacenv.sac_native import NativeSAC
    nat = NativeSAC(gpu, init_seed=0, with_memory=False)
    with pytest.raises(ValueError):
        nat.choose_action(torch.zeros((4, 10), device=gpu))
    batch, noise = _batch(gpu, B=512)
    with pytest.raises(ValueError):
        nat.learn(batch, noise)


@pytest.mark.parametrize("kind", ["native", "torch"])
@pytest.mark.parametrize("optimizer", [False, True])
def test_checkpoint_round_trip_gpu(gpu, built_lib, tmp_path, kind, optimizer):
    """save_models -> load_models into a fresh agent -> learn() bit-identical to the
    original continuing (test_agent_cpu.checkpoint_round_trip); NativeSAC's parameters
    are views of its weights buffer, refreshed by load_models' sync()."""
    from sacenv.agent import VecSAC
    from sacenv.sac_native import NativeSAC
    from test_agent_cpu import checkpoint_round_trip
    cls = NativeSAC if kind == "native" else VecSAC
    checkpoint_round_trip(lambda s: cls(gpu, init_seed=s, with_memory=False), gpu, tmp_path, optimizer)


def test_native_update_network_parameters_refreshes_kernel_copy(gpu, built_lib):
    """A hard target update (tau = 1, as the reference constructor does) after the value
    net changed: the next learn() must see the new target fc2 weights, whose kernel copy
    in fragment order only sync() refreshes."""
    ref, nat = _pair(gpu, seed=6)
    for agent in (ref, nat):
        with torch.no_grad():
            agent.value.fc2.weight.mul_(2.0)
            agent.value.fc2.bias.add_(0.5)
        if agent is nat:
            nat.sync()
        agent.update_network_parameters(tau=1.0)
    batch, noise = _batch(gpu, seed=12)
    lr, ln = ref.learn(batch, noise), nat.learn(batch, noise)
    torch.cuda.synchronize()
    np.testing.assert_allclose([float(x) for x in ln], [float(x) for x in lr], rtol=1e-4)


def test_native_learn_returns_independent_losses(gpu, built_lib):
    _, nat = _pair(gpu, seed=8)
    b1, n1 = _batch(gpu, seed=20)
    b2, n2 = _batch(gpu, seed=21)
    l1 = nat.learn(b1, n1)
    keep = [float(x) for x in l1]
    l2 = nat.learn(b2, n2)
    torch.cuda.synchronize()
    assert [float(x) for x in l1] == keep and [float(x) for x in l2] != keep
