"""sacenv_boat_segment: n_steps BoatEnv.step calls in one persistent launch.

Parity bar: bit-identical to the same number of ``sacenv_boat_step`` launches
(records, terminal obs, the whole arena) -- the per-step kernel is pinned to
the reference by tests/test_gpu_parity.py, so equality carries that parity
over. Covered: open-loop rows, rows behind already-published flags (the
bench's configuration), strided action rows, the pooled transition rows,
every step-kernel instantiation (2/1/0 wind curves, t derived or carried),
refills between segments; the closed loop with the SAC policy handing off per
owner wave (``sacenv.closed_loop.ClosedLoop``) against the eager
``choose_action`` + ``step`` loop (main.py:70-91); a hand-off that never comes.
Reference: environment/boat_env.py:67-126.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _pair(gpu, exp, tmax, dt, N, **kw):
    from sacenv import VecBoatEnv
    cfg = {"base_settings": {"experiment": exp, "test_mode": 0, "t_max": tmax, "dt": dt},
           "boat_env": {"track_width": 30}}
    # the refill is placed by the tests (after every segment), the same for both envs
    kw = dict(dict(seed=11, device=gpu, autoreset=True, max_episode_steps=23, n_helpers=64,
                   auto_refill=False), **kw)
    return VecBoatEnv(cfg, N, **kw), VecBoatEnv(cfg, N, **kw)


@pytest.mark.parametrize("exp,tmax,dt", [(6, 2500.0, 0.25), (4, 20.0, 0.25), (2, 2500.0, 0.25),
                                         (3, 2500.0, 0.25), (6, 20.0, 0.1)])
@pytest.mark.parametrize("flags", ["none", "published"])
def test_segment_equals_steps(exp, tmax, dt, flags, gpu, built_lib):
    N = 777
    a_env, b_env = _pair(gpu, exp, tmax, dt, N)
    nw = a_env.n_pad // 64
    g = torch.Generator(device=gpu)
    g.manual_seed(exp)
    table = torch.rand((300, N), generator=g, device=gpu) * 2 - 1
    table[:, ::7] *= 12.0                      # some rudders break at once
    ready = torch.full((nw,), 0x7FFFFFFF, dtype=torch.int32, device=gpu) if flags == "published" else None
    done = torch.zeros(nw, dtype=torch.int32, device=gpu)
    k = 0
    for rep, K in enumerate((128, 40, 128, 1, 77)):   # crosses refills (period 128)
        rows = table[k % 150: k % 150 + K]          # strided rows of a larger table
        a_env.segment_async(rows, K, act_ready=ready, step_done=done, seq0=k)
        for j in range(K):
            b_env.step_async(rows[j].contiguous())
        a_env.refill()
        b_env.refill()
        k += K
        torch.cuda.synchronize()
        assert torch.equal(a_env.arena, b_env.arena), (rep, K)
        assert int(done.min()) == k and int(done.max()) == k
    a_env.check_status()


@pytest.mark.parametrize("exp", [2, 6])
def test_segment_pooled_rows_equal_step_pooled(exp, gpu, built_lib):
    from sacenv import _lib
    N = 1000
    a_env, b_env = _pair(gpu, exp, 2500.0, 0.25, N)
    row = _lib.trans_bytes(exp) * a_env.n_pad
    K = 50
    acts = torch.rand((K, N), device=gpu) * 2 - 1
    ta = torch.zeros(K * row, dtype=torch.uint8, device=gpu)
    tb = torch.zeros(K * row, dtype=torch.uint8, device=gpu)
    a_env.segment_async(acts, K, trans=ta, trans_stride=row)
    for j in range(K):
        b_env.step_pooled_async(acts[j].contiguous(), tb[j * row:(j + 1) * row])
    torch.cuda.synchronize()
    assert torch.equal(ta, tb)
    assert torch.equal(a_env.arena, b_env.arena)


def test_segment_at_bench_size_equals_steps(gpu, built_lib):
    """65 536 envs, exp 6, 500-step episodes, the bench's refill helpers: two segments."""
    from sacenv import VecBoatEnv
    kw = dict(seed=0, device=gpu, max_episode_steps=500, auto_refill=False)
    cfg = {"base_settings": {"experiment": 6, "test_mode": 0}}
    a_env, b_env = VecBoatEnv(cfg, 65536, **kw), VecBoatEnv(cfg, 65536, **kw)
    a_env.reset()
    b_env.reset()
    acts = torch.rand((256, 65536), device=gpu) * 2 - 1
    ready = torch.full((1024,), 0x7FFFFFFF, dtype=torch.int32, device=gpu)
    for s in range(2):
        a_env.segment_async(acts[128 * s:], 128, act_ready=ready)
        for j in range(128):
            b_env.step_async(acts[128 * s + j])
        a_env.refill()
        b_env.refill()
        torch.cuda.synchronize()
        assert torch.equal(a_env.arena, b_env.arena), s


@pytest.mark.parametrize("exp", [1, 4, 6])
def test_dense_segment_equals_steps(exp, gpu, built_lib):
    """More owner waves than SIMDs (131 072 envs): the segment launch takes the
    two-waves-per-SIMD instantiation (k_rollout_dense, constants as literals and
    scalar registers); bit-identical to step launches, with and without pooled rows."""
    from sacenv import VecBoatEnv, _lib
    from sacenv.closed_loop import occupancy
    N, K = 131072, 64
    kw = dict(seed=3, device=gpu, max_episode_steps=40, auto_refill=False)
    cfg = {"base_settings": {"experiment": exp, "test_mode": 0}}
    a_env, b_env = VecBoatEnv(cfg, N, **kw), VecBoatEnv(cfg, N, **kw)
    o = occupancy(a_env.params, N)
    simds = 4 * torch.cuda.get_device_properties(gpu).multi_processor_count
    if o["seg_grid"] > simds:            # the dense kernel: two owner waves fit per SIMD
        assert o["seg_vgprs"] <= 256 and o["seg_per_cu"] >= 8, o
    a_env.reset()
    b_env.reset()
    acts = torch.rand((2 * K, N), device=gpu) * 2 - 1
    ready = torch.full((N // 64,), 0x7FFFFFFF, dtype=torch.int32, device=gpu)
    row = _lib.trans_bytes(exp) * a_env.n_pad
    ta = torch.zeros(K * row, dtype=torch.uint8, device=gpu)
    tb = torch.zeros_like(ta)
    a_env.segment_async(acts, K, act_ready=ready)
    for j in range(K):
        b_env.step_async(acts[j])
    torch.cuda.synchronize()
    assert torch.equal(a_env.arena, b_env.arena)
    a_env.segment_async(acts[K:], K, act_ready=ready, trans=ta, trans_stride=row)
    for j in range(K):
        b_env.step_pooled_async(acts[K + j].contiguous(), tb[j * row:(j + 1) * row])
    a_env.refill()
    b_env.refill()
    torch.cuda.synchronize()
    assert torch.equal(ta, tb)
    assert torch.equal(a_env.arena, b_env.arena)


@pytest.mark.parametrize("N,K,segs", [(8192, 128, 3), (777, 37, 4)])
def test_closed_loop_equals_eager_loop(N, K, segs, gpu, built_lib):
    """ClosedLoop (the env as segment launches, the SAC policy per step on a second
    stream, handing off per owner wave) = the eager loop of main.py:70-91:
    ``a = choose_action(obs, eps); env.step(a)``, bit for bit (arena and actions)."""
    from sacenv import VecBoatEnv
    from sacenv.closed_loop import ClosedLoop
    from sacenv.sac_native import NativeSAC
    cfg = {"base_settings": {"experiment": 6, "test_mode": 0}}
    kw = dict(seed=5, device=gpu, max_episode_steps=60, n_helpers=256, auto_refill=False)
    a_env, b_env = VecBoatEnv(cfg, N, **kw), VecBoatEnv(cfg, N, **kw)
    a_env.reset()
    b_env.reset()
    agent = NativeSAC(gpu, init_seed=3, with_memory=False)
    loop = ClosedLoop(a_env, agent, segment=K, handoff=True)
    g = torch.Generator(device=gpu)
    g.manual_seed(1)
    eps = torch.randn((segs, K, N), generator=g, device=gpu)
    acts_b = []
    for s in range(segs):
        loop.run(eps[s])
        for k in range(K):
            a = agent.choose_action(b_env.obs, eps=eps[s, k])
            acts_b.append(a.reshape(-1))
            b_env.step_async(a.reshape(-1).contiguous())
        a_env.refill()
        b_env.refill()
        torch.cuda.synchronize()
        if not torch.equal(loop.actions[:K], torch.stack(acts_b[-K:])):
            nz = [(loop.actions[k] != 0).sum().item() for k in range(min(K, 6))]
            raise AssertionError(
                f"segment {s}: actions differ; rows nonzero {nz}, status {int(a_env.status[1])}, step_done "
                f"{sorted(set(loop.step_done.tolist()))[:6]}, act_ready {sorted(set(loop.act_ready.tolist()))[:6]}, "
                f"plan {loop.plan}")
        assert torch.equal(a_env.arena, b_env.arena), s
    a_env.check_status()
    assert int(a_env.status[1]) == 0
    assert int(loop.step_done.min()) == segs * K and int(loop.act_ready.max()) == segs * K


def test_closed_loop_run_eager_equals_run(gpu, built_lib):
    """``ClosedLoop.run_eager`` (choose_action then one step launch per step, one
    stream: the form bench.py --closed-loop reports when the policy dominates) and
    the hand-off ``run`` give the same arena, bit for bit."""
    from sacenv import VecBoatEnv
    from sacenv.closed_loop import ClosedLoop
    from sacenv.sac_native import NativeSAC
    N, K, segs = 8192, 64, 2
    cfg = {"base_settings": {"experiment": 6, "test_mode": 0}}
    kw = dict(seed=9, device=gpu, max_episode_steps=50, n_helpers=256, auto_refill=False)
    a_env, b_env = VecBoatEnv(cfg, N, **kw), VecBoatEnv(cfg, N, **kw)
    a_env.reset()
    b_env.reset()
    agent = NativeSAC(gpu, init_seed=4, with_memory=False)
    la, lb = ClosedLoop(a_env, agent, segment=K, handoff=True), ClosedLoop(b_env, agent, segment=K)
    assert lb.plan is None and not lb.handoff      # no co-residency plan, no exclusive queue
    with pytest.raises(RuntimeError):
        lb.run_handoff(torch.zeros((1, b_env.num_envs), device=gpu))
    g = torch.Generator(device=gpu)
    g.manual_seed(2)
    eps = torch.randn((segs, K, N), generator=g, device=gpu)
    for s in range(segs):
        la.run(eps[s])
        lb.run(eps[s])          # the default form: eager
        a_env.refill()
        b_env.refill()
        torch.cuda.synchronize()
        assert torch.equal(a_env.arena, b_env.arena), s
    la.check()


def test_segment_handoff_timeout_sets_status(gpu, built_lib):
    """A row whose flag never comes: the launch gives up after ~seconds of polling,
    flags SACENV_STATUS_HANDOFF_TIMEOUT and returns (no hang)."""
    from sacenv import VecBoatEnv, _lib
    env = VecBoatEnv({"base_settings": {"experiment": 1}}, 128, device=gpu, autoreset=False)
    env.reset()
    ready = torch.zeros(2, dtype=torch.int32, device=gpu)
    ready[0] = 3                                     # wave 0: rows 0..2 published, wave 1: none
    acts = torch.zeros((8, 128), device=gpu)
    env.segment_async(acts, 8, act_ready=ready)
    torch.cuda.synchronize()
    assert int(env.status[1]) & _lib.STATUS_HANDOFF_TIMEOUT
    assert int(env.index[0]) == 3 and int(env.index[64]) == 0


def test_closed_loop_after_a_timeout_refuses_and_steps_nothing(gpu, built_lib):
    """after a hand-off timeout, later closed-loop launches must not step
    on stale rows. The device's abort protocol makes them no-ops (no hang), check()
    and check_status() raise, and run() refuses once check() has seen it."""
    from sacenv import VecBoatEnv, _lib
    from sacenv.closed_loop import ClosedLoop
    from sacenv.sac_native import NativeSAC
    env = VecBoatEnv({"base_settings": {"experiment": 1}}, 128, device=gpu, autoreset=False)
    env.reset()
    agent = NativeSAC(gpu, init_seed=3, with_memory=False)
    loop = ClosedLoop(env, agent, segment=8, handoff=True)
    ready = torch.zeros(2, dtype=torch.int32, device=gpu)
    ready[0] = 3                                      # wave 1's rows never come: timeout
    env.segment_async(torch.zeros((8, 128), device=gpu), 8, act_ready=ready)
    torch.cuda.synchronize()
    assert int(env.status[1]) & _lib.STATUS_HANDOFF_TIMEOUT
    before = env.arena.clone()
    loop.run(torch.randn((4, 128), device=gpu))      # enqueued: the device refuses it
    torch.cuda.synchronize()
    assert torch.equal(env.arena, before)            # nothing stepped, nothing written
    assert int(loop.step_done.min()) == _lib.FLAG_ABORT - 2**32   # (int32 view of the abort flag)
    with pytest.raises(_lib.SacenvError):
        loop.check()
    with pytest.raises(_lib.SacenvError):
        loop.run(torch.randn((4, 128), device=gpu))
    with pytest.raises(_lib.SacenvError):
        env.check_status()


def test_closed_loop_at_the_largest_co_resident_size(gpu, built_lib):
    """the co-residency plan from both kernels' VGPRs and LDS (the
    library's hipFuncGetAttributes); at the largest env count it admits -- the bench's
    65 536, one owner wave per SIMD beside one lean policy wave -- the closed loop
    equals the eager loop bit for bit; one owner wave more is refused."""
    from sacenv import VecBoatEnv
    from sacenv.closed_loop import ClosedLoop, make_plan, occupancy
    from sacenv.sac_native import NativeSAC
    cfg = {"base_settings": {"experiment": 6, "test_mode": 0}}
    kw = dict(seed=5, device=gpu, max_episode_steps=40, n_helpers=2048, auto_refill=False)
    probe = VecBoatEnv(cfg, 64, **kw)
    cus = torch.cuda.get_device_properties(gpu).multi_processor_count
    o = occupancy(probe.params, 64)
    print(f"kernels: {o}, {cus} CUs")
    N = make_plan(cus, 1, o["seg_vgprs"], o["seg_lds"], 1, o["act_vgprs"], o["act_lds"]).max_envs
    print(f"largest closed loop: {N} envs")
    assert N >= 65536                                 # the bench's size runs closed loop
    with pytest.raises(ValueError):
        make_plan(cus, N // 64 + 1, o["seg_vgprs"], o["seg_lds"], N // 64 + 1, o["act_vgprs"], o["act_lds"], N + 64)
    a_env, b_env = VecBoatEnv(cfg, N, **kw), VecBoatEnv(cfg, N, **kw)
    a_env.reset()
    b_env.reset()
    agent = NativeSAC(gpu, init_seed=3, with_memory=False)
    K = 16
    g = torch.Generator(device=gpu)
    g.manual_seed(1)
    with ClosedLoop(a_env, agent, segment=K, handoff=True) as loop:   # releases its queue on exit
        for s in range(2):
            eps = torch.randn((K, N), generator=g, device=gpu)
            loop.run(eps)
            for k in range(K):
                b_env.step_async(agent.choose_action(b_env.obs, eps=eps[k]).reshape(-1).contiguous())
            a_env.refill()
            b_env.refill()
            torch.cuda.synchronize()
            assert torch.equal(a_env.arena, b_env.arena), s
        loop.check()
    assert loop._policy_handle is None


def test_closed_loop_survives_shared_hardware_queues(gpu, built_lib):
    """Ordinary HIP streams are spread over GPU_MAX_HW_QUEUES shared hardware queues; a
    policy stream that landed on the env stream's queue serialised the two and
    deadlocked the hand-off until its timeout (seen in the full GPU suite). The policy
    stream now has a queue of its own (sacenv_stream_create_exclusive): with many
    streams created and used first, every loop still equals the eager loop."""
    from sacenv import VecBoatEnv
    from sacenv.closed_loop import ClosedLoop
    from sacenv.sac_native import NativeSAC
    streams = [torch.cuda.Stream(device=gpu) for _ in range(9)]
    for s in streams:
        with torch.cuda.stream(s):
            torch.ones(16, device=gpu).sum()
    cfg = {"base_settings": {"experiment": 6, "test_mode": 0}}
    kw = dict(seed=9, device=gpu, max_episode_steps=50, n_helpers=256, auto_refill=False)
    agent = NativeSAC(gpu, init_seed=4, with_memory=False)
    N, K = 4096, 64
    g = torch.Generator(device=gpu)
    g.manual_seed(2)
    for trial in range(5):
        a_env, b_env = VecBoatEnv(cfg, N, **kw), VecBoatEnv(cfg, N, **kw)
        a_env.reset()
        b_env.reset()
        loop = ClosedLoop(a_env, agent, segment=K, handoff=True)
        eps = torch.randn((K, N), generator=g, device=gpu)
        loop.run(eps)
        for k in range(K):
            b_env.step_async(agent.choose_action(b_env.obs, eps=eps[k]).reshape(-1).contiguous())
        torch.cuda.synchronize()
        loop.check()
        assert torch.equal(a_env.arena, b_env.arena), trial
        extra = torch.cuda.Stream(device=gpu)   # shift the round-robin for the next trial
        with torch.cuda.stream(extra):
            torch.ones(16, device=gpu).sum()
        streams.append(extra)
