"""GPU parity: the HIP engine vs the reference's fixtures and the CPU oracle.

Bar (BASELINE.json north_star): done/termination codes bit-exact, float64
state within STATE_TOL = 1e-5 of the CPU reference for identical seeds.
Observations are float32 outputs: compared within f32 rounding of the
reference's float64 values (OBS_TOL). RNG draws (start y, knot values) are
compared bit-exactly.
"""
import numpy as np
import pytest
import torch

from boat_oracle import OracleConfig, OracleVecBoat, config_from_fixture
from conftest import golden, seeded_fixtures

pytestmark = pytest.mark.gpu

STATE_TOL = 1e-5
OBS_TOL = 1e-6
STATE_KEYS = ("s_x", "s_y", "s_r", "v_x", "v_y", "v_r", "a_x", "a_y", "a_r",
              "rudder_angle", "t", "fuel", "index")


def _cfg_dict(z):
    c = config_from_fixture(z)
    return {"base_settings": {"experiment": c.experiment, "test_mode": c.test_mode,
                              "dt": c.dt, "t_max": c.t_max},
            "boat_env": {"track_width": c.track_width, "goal_line": c.goal_line,
                         "boat_out_of_bounds_offset": c.oob_offset},
            "boat": {"fuel": c.fuel}}


def _state_matrix(env):
    d = env.state_dict()
    d["rudder_angle"] = d["rudder"]
    return np.stack([np.asarray(d[k], np.float64) for k in STATE_KEYS], 1)


@pytest.mark.parametrize("name", seeded_fixtures())
def test_seeded_fixture_explicit_reset(name, gpu, built_lib):
    """Step the reference's seeded runs; reset ended envs via reset(ids)."""
    from sacenv import VecBoatEnv
    z = golden(name)
    E, S = z["reward"].shape
    env = VecBoatEnv(_cfg_dict(z), E, seeds=z["seeds"], device=gpu, autoreset=False,
                     record_knots=True, record_accel=True, record_reward64=True)
    obs = env.reset().cpu().numpy()
    np.testing.assert_allclose(obs, z["init_obs"], rtol=0, atol=OBS_TOL)
    np.testing.assert_array_equal(env.start_y.cpu().numpy(), z["init_start_y"])
    worst = 0.0
    for k in range(S):
        a = torch.from_numpy(np.ascontiguousarray(z["actions"][:, k])).to(gpu)
        o, r, d, info = env.step(a)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(info["term"].cpu().numpy(), z["term"][:, k], err_msg=f"{k}")
        np.testing.assert_array_equal(d.cpu().numpy(), z["done"][:, k], err_msg=f"{k}")
        st = _state_matrix(env)
        err = np.abs(st - z["state"][:, k]).max()
        worst = max(worst, err)
        assert err <= STATE_TOL, f"state off by {err} at step {k}"
        np.testing.assert_allclose(o.cpu().numpy(), z["obs"][:, k], rtol=OBS_TOL, atol=OBS_TOL)
        np.testing.assert_allclose(env.reward64.cpu().numpy(), z["reward"][:, k], rtol=0,
                                   atol=STATE_TOL)
        ended = np.flatnonzero(z["done"][:, k])
        if ended.size:
            np.testing.assert_allclose(info["final_ep_reward"].cpu().numpy()[ended],
                                       z["ep_reward"][ended, k], rtol=0, atol=1e-4)
            ro = env.reset(ended).cpu().numpy()
            torch.cuda.synchronize()
            np.testing.assert_allclose(ro[ended], z["reset_obs"][ended, k], rtol=0, atol=OBS_TOL)
            np.testing.assert_array_equal(env.start_y.cpu().numpy()[ended], z["start_y"][ended, k])
    np.testing.assert_array_equal(env.counters.cpu().numpy().T, z["counters"])
    print(f"{name}: worst state err {worst:.3e}")


@pytest.mark.parametrize("name", ["seeded_exp6_uniform.npz", "seeded_exp3_big.npz",
                                  "seeded_exp6_fuel.npz", "seeded_exp6_narrow.npz"])
def test_seeded_fixture_autoreset(name, gpu, built_lib):
    """In-kernel auto-reset: obs row = new episode's obs, final_obs = terminal obs."""
    from sacenv import VecBoatEnv
    z = golden(name)
    E, S = z["reward"].shape
    env = VecBoatEnv(_cfg_dict(z), E, seeds=z["seeds"], device=gpu, autoreset=True,
                     record_accel=True, n_helpers=4)
    env.reset()
    for k in range(S):
        a = torch.from_numpy(np.ascontiguousarray(z["actions"][:, k])).to(gpu)
        o, r, d, info = env.step(a)
        torch.cuda.synchronize()
        done = z["done"][:, k].astype(bool)
        np.testing.assert_array_equal(info["term"].cpu().numpy(), z["term"][:, k])
        o = o.cpu().numpy()
        np.testing.assert_allclose(o[~done], z["obs"][~done, k], rtol=OBS_TOL, atol=OBS_TOL)
        if done.any():
            fo = info["final_obs"].cpu().numpy()
            np.testing.assert_allclose(fo[done], z["obs"][done, k], rtol=OBS_TOL, atol=OBS_TOL)
            np.testing.assert_allclose(o[done], z["reset_obs"][done, k], rtol=0, atol=OBS_TOL)
            np.testing.assert_array_equal(env.start_y.cpu().numpy()[done], z["start_y"][done, k])
        st = _state_matrix(env)
        live = ~done
        assert np.abs(st[live] - z["state"][live, k]).max(initial=0) <= STATE_TOL
    np.testing.assert_array_equal(env.counters.cpu().numpy().T, z["counters"])


@pytest.mark.parametrize("name", ["wind_exp4.npz", "wind_exp5.npz", "wind_exp6.npz",
                                  "wind_exp6_tmax5.npz"])
def test_wind_tables_vs_reference(name, gpu, built_lib):
    """GPU wind curves vs the reference's interp1d tables (wind.py:69-99)."""
    from sacenv import VecBoatEnv
    z = golden(name)
    exp, L = int(z["experiment"]), int(z["L"])
    n = len(z["seeds"])
    env = VecBoatEnv({"base_settings": {"experiment": exp, "t_max": L * 0.25}}, n,
                     seeds=z["seeds"], device=gpu)
    np.testing.assert_array_equal(env.start_y.cpu().numpy(), z["start_y"])
    idx = z["idx"]
    ids = np.repeat(np.arange(n, dtype=np.int32), len(idx))
    ix = np.tile(idx.astype(np.int32), n)
    v, a = env.wind_eval(ids, ix)
    torch.cuda.synchronize()
    v = v.cpu().numpy().reshape(n, len(idx))
    a = a.cpu().numpy().reshape(n, len(idx))
    np.testing.assert_allclose(v, z["vel"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(a, z["ang"], rtol=0, atol=1e-12)


def test_wind_tables_span_their_range_at_scale(gpu, built_lib):
    """wind.py:86-99's min-max renormalisation makes a renormalised curve's extreme
    samples exactly 0 and 1 (x max_velocity for the speed, x 2 pi for the angle). The
    fit finds the grid extrema from the cubic's critical points and folds them into
    the knots; over 2 048 exp-6 episodes (full 10 000-sample tables through
    sacenv_boat_wind_eval) every table stays inside its range, and every curve's
    extreme sample lands on the range's ends within a few ulp."""
    from sacenv import VecBoatEnv
    n, L = 2048, 10000
    env = VecBoatEnv({"base_settings": {"experiment": 6}}, n, seed=41, device=gpu, autoreset=False)
    ids = torch.arange(n, dtype=torch.int32, device=gpu).repeat_interleave(L)
    ix = torch.arange(L, dtype=torch.int32, device=gpu).repeat(n)
    v, a = env.wind_eval(ids, ix)
    v, a = v.view(n, L), a.view(n, L)
    for t, top in ((v, float(env.cfg.max_velocity)), (a, 2 * np.pi)):
        lo, hi = t.min(1).values.cpu().numpy(), t.max(1).values.cpu().numpy()
        eps = 8 * np.finfo(np.float64).eps * top
        assert (lo >= -eps).all() and (hi <= top + eps).all(), (lo.min(), hi.max())
        # a renormalised curve (its raw spline left [0, 1]) touches BOTH ends; a curve
        # that was not renormalised touches neither (its raw samples lie strictly inside)
        at_lo, at_hi = lo <= eps, hi >= top - eps
        assert np.array_equal(at_lo, at_hi), (np.flatnonzero(at_lo != at_hi)[:5], lo, hi)
        assert at_lo.sum() > n // 4


@pytest.mark.parametrize("autoreset", [False, True])
def test_rng_draws_bit_exact_across_many_resets(autoreset, gpu, built_lib):
    """Knots/start-y of 150 consecutive Boats per env == numpy RandomState (crosses
    many 624-word MT blocks, incl. windows straddling a block end). In autoreset
    mode the draws happen up to 128 episodes ahead; the sequence is the same."""
    from sacenv import VecBoatEnv
    seeds = np.array([0, 5, 99, 2**32 - 1], np.uint64)
    env = VecBoatEnv({"base_settings": {"experiment": 6}}, len(seeds), seeds=seeds, device=gpu,
                     record_knots=True, autoreset=autoreset, n_helpers=3)
    rs = [np.random.RandomState(int(s)) for s in seeds]
    for r in range(150):
        if r > 0:
            env.reset()
        torch.cuda.synchronize()
        kn = env.knots_raw.cpu().numpy()       # [2, 8, E]
        sy = env.start_y.cpu().numpy()
        for e, g in enumerate(rs):
            assert sy[e] == g.randint(-640, 640), (r, e)
            assert np.array_equal(kn[0, :, e], g.random_sample(8)), (r, e)
            assert np.array_equal(kn[1, :, e], g.random_sample(8)), (r, e)
    if not autoreset:   # the device MT state is numpy's state
        key = env.mt_key.cpu().numpy().view(np.uint32)
        for e, g in enumerate(rs):
            st = g.get_state()
            pos = int(env.mt_pos[e]) & 0xFFFF
            if pos == st[2]:
                assert np.array_equal(key[e], st[1])
            else:   # block exhausted: numpy twists lazily, the device may have already
                assert pos == 0 and st[2] == 624


def test_refill_twists_the_next_mt_block_ahead(gpu, built_lib):
    """After every refill each env's mt_next is the block numpy's MT19937 generates after
    mt_key (mt_pos bit 16 set, the index back inside the current block), including envs
    whose draws ran past the block end into mt_next (the refill's draw launch reads on
    there; its fit launch makes it current and twists the next). The draws themselves
    are pinned by test_rng_draws_bit_exact_across_many_resets and the bench-path tests."""
    from sacenv import VecBoatEnv
    n = 512
    env = VecBoatEnv({"base_settings": {"experiment": 6}}, n, seed=11, device=gpu, autoreset=True)
    g = torch.Generator(device="cpu").manual_seed(3)
    acts = (torch.rand(256, n, generator=g) * 2 - 1).to(gpu)
    wrapped = 0
    for seg in range(8):
        p0 = env.mt_pos.clone() & 0xFFFF
        env.segment_async(acts, 256)
        env.refill()
        torch.cuda.synchronize()
        mp = env.mt_pos.clone()
        pos = mp & 0xFFFF
        assert bool(((mp >> 16) & 1).all()) and int(pos.max()) <= 624, seg
        assert torch.equal(env.mt_index, pos)   # the masked accessor (mt_pos is the raw word)
        wrapped += int((pos < p0).sum())
        key = env.mt_key.cpu().numpy().view(np.uint32)
        nxt = env.mt_next.cpu().numpy().view(np.uint32)
        for e in range(seg, n, 29):
            rs = np.random.RandomState()
            rs.set_state(("MT19937", key[e].copy(), 624, 0, 0.0))
            rs.bytes(4)   # one word: numpy twists the block first
            assert np.array_equal(rs.get_state()[1], nxt[e]), (seg, e)
    assert wrapped > 0   # some envs' draws did cross into mt_next


def test_spline_g_on_device(gpu, built_lib):
    from sacenv import VecBoatEnv
    from sacenv.config import spline_g
    for nk in (4, 8, 16):
        env = VecBoatEnv({"base_settings": {"experiment": 6}, "wind": {"fixed_points": nk}}, 2,
                         device=gpu)
        torch.cuda.synchronize()
        np.testing.assert_allclose(env.spline_g.cpu().numpy(), spline_g(nk), rtol=0, atol=1e-15)


def test_autoreset_every_step_one_step_episodes(gpu, built_lib):
    """|action| > 10.5 breaks the rudder on the first step: every env ends in every
    launch, the worst case for the slot ring (REFILL_PERIOD = 256 episodes consumed
    between two refills, then 256 drawn per env by one refill). Draws must stay exact."""
    from sacenv import VecBoatEnv
    E, S = 70, 270
    seeds = np.arange(E, dtype=np.uint64) * 7 + 3
    env = VecBoatEnv({"base_settings": {"experiment": 6, "test_mode": 0}}, E, seeds=seeds,
                     device=gpu, autoreset=True, n_helpers=5, record_knots=True)
    ora = OracleVecBoat(OracleConfig(experiment=6), seeds)
    acts = np.full(E, 20.0, np.float32)
    for k in range(S):
        o, r, d, info = env.step(torch.from_numpy(acts).to(gpu))
        ro = ora.step(acts)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(info["term"].cpu().numpy(), ro["term"])
        assert (ro["term"] == 4).all()
        np.testing.assert_allclose(o.cpu().numpy(), ro["reset_obs"], rtol=OBS_TOL, atol=OBS_TOL)
        np.testing.assert_allclose(info["final_obs"].cpu().numpy(), ro["obs"], rtol=OBS_TOL,
                                   atol=OBS_TOL)
        np.testing.assert_array_equal(env.start_y.cpu().numpy(), ora.start_y)
        np.testing.assert_array_equal(env.knots_raw.cpu().numpy().transpose(2, 0, 1), ora.knots)
    env.check_status()


@pytest.mark.parametrize("period", [1, 7, 32])
def test_refill_schedule_any_period_within_the_ring(period, gpu, built_lib):
    """Refills placed by hand (auto_refill off) every `period` steps, once doubled,
    give the same episodes as the oracle; a ring that runs dry sets the status bit."""
    from sacenv import VecBoatEnv, _lib
    E = 130
    seeds = np.arange(E, dtype=np.uint64) * 3 + 11
    cfg = {"base_settings": {"experiment": 6, "test_mode": 0}}
    env = VecBoatEnv(cfg, E, seeds=seeds, device=gpu, autoreset=True, n_helpers=16,
                     record_knots=True, auto_refill=False, max_episode_steps=3)
    ora = OracleVecBoat(OracleConfig(experiment=6), seeds, max_episode_steps=3)
    rng = np.random.default_rng(period)
    for k in range(96):
        a = rng.uniform(-1, 1, E).astype(np.float32)
        if k % 5 == 0:
            a[: E // 2] = 20.0      # half the envs end at once
        o, r, d, info = env.step(torch.from_numpy(a).to(gpu))
        ro = ora.step(a)
        if (k + 1) % period == 0:
            env.refill()
            if k == 40:
                env.refill()        # back to back: harmless
        torch.cuda.synchronize()
        np.testing.assert_array_equal(info["term"].cpu().numpy(), ro["term"], err_msg=f"{k}")
        np.testing.assert_allclose(o.cpu().numpy(), ro["reset_obs"], rtol=OBS_TOL, atol=OBS_TOL)
        np.testing.assert_array_equal(env.knots_raw.cpu().numpy().transpose(2, 0, 1), ora.knots)
    env.check_status()
    # no refill for more than REFILL_PERIOD launches of one-step episodes: flagged
    dry = VecBoatEnv(cfg, 64, seed=1, device=gpu, autoreset=True, auto_refill=False, n_helpers=4)
    for _ in range(_lib.REFILL_PERIOD + 1):
        dry.step(torch.full((64,), 20.0, device=gpu))
    dry.refill()
    with pytest.raises(_lib.SacenvError):
        dry.check_status()


@pytest.mark.parametrize("exp", [1, 2, 3, 4, 5, 6])
def test_recorded_episode_replay(exp, gpu, built_lib):
    """The reference's own recorded episodes (4 959 / 4 963 steps, goal reached)."""
    from sacenv import VecBoatEnv
    z = golden(f"recorded_exp{exp}.npz")
    tr = z["trace"]
    cols = [str(c) for c in z["columns"]]
    c = {n: cols.index(n) for n in cols}
    table = np.stack([z["wind_velocity"], z["wind_angle"]])
    env = VecBoatEnv({"base_settings": {"experiment": exp, "test_mode": 1}}, 1, device=gpu,
                     autoreset=False, wind_table=table, record_reward64=True)
    env.reset_explicit([0], [int(tr[0, c["boat_position_y"]])])
    n = len(tr) - 1
    act = torch.zeros(1, dtype=torch.float32, device=gpu)
    hist = []
    for k in range(n + 1):
        env.step(act)
        hist.append(torch.stack([env.s_x, env.s_y, env.v_x, env.v_y, env.s_r]).clone())
    torch.cuda.synchronize()
    h = torch.cat(hist, 1).cpu().numpy().T       # [n+1, 5]
    ref = tr[1:, [c["boat_position_x"], c["boat_position_y"], c["boat_velocity_x"],
                  c["boat_velocity_y"], c["boat_angle"]]]
    err = np.abs(h[:n] - ref).max()
    assert err <= STATE_TOL, err
    assert int(env.term[0]) == 1                 # reached_goal on the last step
    if exp == 6:
        assert abs(float(env.ep_reward[0]) - float(z["episode_reward"])) < 1e-6


def test_full_size_subsample_vs_oracle(gpu, built_lib):
    """65 536 envs (the bench config) with auto-reset and 500-step truncation:
    envs are independent, so a random subset is checked against the oracle
    run on just those seeds."""
    from sacenv import VecBoatEnv
    N, S = 65536, 120
    rng = np.random.default_rng(1)
    seeds = np.arange(N, dtype=np.uint64) + 1000
    env = VecBoatEnv({"base_settings": {"experiment": 6, "test_mode": 0}}, N, seeds=seeds,
                     device=gpu, autoreset=True, max_episode_steps=50)
    env.reset()
    pick = np.sort(rng.choice(N, 256, replace=False))
    ora = OracleVecBoat(OracleConfig(experiment=6), seeds[pick], max_episode_steps=50)
    ora.reset()
    acts = rng.uniform(-1, 1, (S, N)).astype(np.float32)
    acts_d = torch.from_numpy(acts).to(gpu)
    n_trunc = 0
    for k in range(S):
        o, r, d, info = env.step(acts_d[k])
        ro = ora.step(acts[k, pick])
        torch.cuda.synchronize()
        term = info["term"].cpu().numpy()[pick]
        np.testing.assert_array_equal(term, ro["term"], err_msg=f"step {k}")
        np.testing.assert_allclose(o.cpu().numpy()[pick], ro["reset_obs"], rtol=OBS_TOL,
                                   atol=OBS_TOL)
        n_trunc += int((term == 6).sum())
        sx = env.s_x.cpu().numpy()[pick]
        assert np.abs(sx - ora.s_x).max() <= STATE_TOL
    assert n_trunc > 0


SHIM_FIELDS = ("s_x", "s_y", "s_r", "v_x", "v_y", "v_r", "a_x", "a_y", "a_r", "rudder_angle", "t", "fuel", "index")


def _shim_state(env):
    """The fixture's 13 state fields read through the drop-in's env.boat (boat_env.py:143-306)."""
    b = env.boat
    return np.array([getattr(b, f) for f in SHIM_FIELDS], np.float64)


def test_dropin_boatenv_shares_global_rng(gpu, built_lib):
    """BoatEnv shim driven like main.py:70-91 reproduces the seeded reference run --
    all 13 state fields through env.boat.* and the obs, every step, the state after
    every reset -- and leaves numpy's global stream exactly where the reference would."""
    from sacenv import BoatEnv
    z = golden("seeded_exp6_uniform.npz")
    assert tuple(str(f) for f in z["state_fields"]) == SHIM_FIELDS
    e = 1
    np.random.seed(int(z["seeds"][e]))
    env = BoatEnv(_cfg_dict(z), None, device=gpu)
    obs = env.reset()
    np.testing.assert_allclose(obs, z["init_obs"][e], atol=OBS_TOL)
    np.testing.assert_allclose(_shim_state(env), z["init_state"][e], rtol=0, atol=STATE_TOL)
    assert env.action_space.shape == (1,) and env.observation_space.shape == (11,)
    S = z["reward"].shape[1]
    resets = 0
    for k in range(S):
        o, r, d, info = env.step(np.array([z["actions"][e, k]], np.float32))
        assert d == bool(z["done"][e, k])
        np.testing.assert_allclose(_shim_state(env), z["state"][e, k], rtol=0, atol=STATE_TOL,
                                   err_msg=f"step {k}")
        np.testing.assert_allclose(o, z["obs"][e, k], rtol=0, atol=OBS_TOL, err_msg=f"step {k}")
        assert abs(r - z["reward"][e, k]) <= STATE_TOL
        assert abs(info["episode_reward"] - z["ep_reward"][e, k]) <= STATE_TOL
        assert info is env.info
        if d:
            assert info["termination"] == "rudder_broken"
            ro = env.reset()
            assert env.info["episode_reward"] == 0
            np.testing.assert_allclose(ro, z["reset_obs"][e, k], rtol=0, atol=OBS_TOL)
            np.testing.assert_allclose(_shim_state(env), z["reset_state"][e, k], rtol=0, atol=STATE_TOL)
            assert env.boat.s_y_start == int(z["start_y"][e, k])
            resets += 1
    assert resets > 0
    ora = OracleVecBoat(OracleConfig(experiment=6), z["seeds"][e:e + 1])
    ora.reset()
    for k in range(S):
        ro = ora.step(z["actions"][e:e + 1, k])
    assert np.random.random_sample() == ora.rngs[0].random_sample()
    row = env.return_all_data()
    assert set(row) == {"boat_position_x", "boat_position_y", "boat_velocity_x",
                        "boat_velocity_y", "boat_angle", "action_rudder", "reward",
                        "rudder_angle", "n"}
    assert len(env.boat.wind.wind_velocity) == 10000


def test_dropin_boatenv_long_reference_run(gpu, built_lib):
    """The drop-in over 10 000 steps of a recorded reference run (long_exp6.npz env 1:
    the U-turn program, episodes ended by s_x < 0 and the default-t_max timeout), driven
    as main.py:70-91 drives the reference: one step() per action, reset() when done
    (numpy's global stream draws the next Boat). Every step: done, termination and
    reward; at the kept steps: the 13 state fields through env.boat.* and the obs, and
    after each reset the fresh Boat."""
    from sacenv import BoatEnv
    z = golden("long_exp6.npz")
    keep = {int(k): j for j, k in enumerate(z["keep"])}
    e = 1
    np.random.seed(int(z["seeds"][e]))
    env = BoatEnv(_cfg_dict(z), None, device=gpu)
    obs = env.reset()
    np.testing.assert_allclose(obs, z["init_obs"][e], atol=OBS_TOL)
    names = {v: k for k, v in {"reached_goal": 1, "out_of_bounds": 2, "out_of_fuel": 3, "rudder_broken": 4,
                               "timeout": 5}.items()}
    S = int(z["n_steps"])
    ends = 0
    for k in range(S):
        o, r, d, info = env.step(np.array([z["actions"][e, k]], np.float32))
        assert d == bool(z["done"][e, k]), f"step {k}"
        assert abs(r - z["reward"][e, k]) <= STATE_TOL, f"step {k}"
        j = keep.get(k)
        if j is not None:
            np.testing.assert_allclose(_shim_state(env), z["state"][e, j], rtol=0, atol=STATE_TOL,
                                       err_msg=f"step {k}")
            np.testing.assert_allclose(o, z["obs"][e, j], rtol=0, atol=OBS_TOL, err_msg=f"step {k}")
        if d:
            assert info["termination"] == names[int(z["term"][e, k])], f"step {k}"
            ro = env.reset()
            np.testing.assert_allclose(ro, z["reset_obs"][e, j], rtol=0, atol=OBS_TOL)
            np.testing.assert_allclose(_shim_state(env), z["reset_state"][e, j], rtol=0, atol=STATE_TOL)
            ends += 1
    assert ends == int(z["done"][e].sum()) > 0
    assert [env.info[n] for n in ("reached_goal", "out_of_bounds", "out_of_fuel", "rudder_broken",
                                  "timeout")] == [int(c) for c in z["counters"][e]]


def test_bad_config_raises(gpu, built_lib):
    from sacenv import VecBoatEnv
    with pytest.raises(ValueError):
        VecBoatEnv({"base_settings": {"experiment": 7}}, 4, device=gpu)
    with pytest.raises(ValueError):
        VecBoatEnv({"base_settings": {"experiment": 6}, "wind": {"fixed_points": 3}}, 4, device=gpu)


def test_step_async_refuses_bad_action_tensors(gpu, built_lib):
    """The kernel reads num_envs f32 values: wrong dtype, length, layout or device
    raise before the launch instead of reading out of bounds."""
    from sacenv import VecBoatEnv
    env = VecBoatEnv({"base_settings": {"experiment": 6}}, 100, device=gpu)
    env.step_async(torch.zeros(100, device=gpu))
    for bad in (torch.zeros(99, device=gpu), torch.zeros(100, device=gpu, dtype=torch.float64),
                torch.zeros(200, device=gpu)[::2], torch.zeros(100)):
        with pytest.raises(ValueError):
            env.step_async(bad)
    with pytest.raises(TypeError):
        env.step_async([0.0] * 100)


# ---------------------------------------------------------------- toy envs (A17, A18)

def _toy_env(kind, n, **kw):
    from sacenv.toys import CarEnv, ParachuteEnv
    return (ParachuteEnv if kind == 1 else CarEnv)(num_envs=n, device="cuda", **kw)


@pytest.mark.parametrize("kind,name,tol", [(1, "toy_parachute.npz", 0.0), (2, "toy_car.npz", 1e-5)])
def test_toy_env_reproduces_reference_script(kind, name, tol, gpu, built_lib):
    """Every env replays the reference script's recorded signals; the loop ends where the
    script's does (parachute: ground at iteration 2654; car: t > t_max at 5000)."""
    sig = golden(name)["signals"]                     # [n_signals, iterations - 1]
    n_rec = sig.shape[1]
    env = _toy_env(kind, 100, autoreset=False)
    rows, terms = [], []
    for k in range(n_rec + 2):
        env.step()
        rows.append(env.state.clone())
        terms.append(env.term.clone())
    torch.cuda.synchronize()
    st = torch.stack(rows).cpu().numpy()              # [steps, 5, N]
    tm = torch.stack(terms).cpu().numpy()             # [steps, N]
    cols = [1] if kind == 1 else [2, 3]
    got = st[1:n_rec + 1][:, cols, :]                 # iterations 2 .. n_rec+1
    want = sig.T[:, :, None]
    np.testing.assert_allclose(got, np.broadcast_to(want, got.shape), rtol=0, atol=tol)
    assert (tm[:n_rec] == 0).all()
    end_term = 1 if kind == 1 else 5                  # ground / timeout
    end_step = n_rec + 1 if kind == 1 else n_rec      # parachute breaks before recording
    assert (tm[end_step] == end_term).all(), tm[end_step - 1: end_step + 2, :3]


@pytest.mark.parametrize("kind", [1, 2])
def test_toy_autoreset_vs_oracle(kind, gpu, built_lib):
    from toy_oracle import OracleToy
    N, T = 1000, 150
    env = _toy_env(kind, N, autoreset=True, max_episode_steps=37)
    ora = OracleToy(kind, N, max_episode_steps=37, autoreset=True)
    np.testing.assert_array_equal(env.obs.cpu().numpy(), ora.reset())
    for k in range(T):
        env.step()
        r = ora.step()
        np.testing.assert_array_equal(env.term.cpu().numpy(), r["term"], err_msg=f"step {k}")
        np.testing.assert_array_equal(env.done.cpu().numpy().astype(bool), r["done"])
        np.testing.assert_allclose(env.obs.cpu().numpy(), r["obs"], rtol=1e-6, atol=1e-5)
        np.testing.assert_allclose(env.state.cpu().numpy(), r["state"], rtol=0, atol=1e-5)
        d = r["done"]
        if d.any():
            np.testing.assert_allclose(env.final_obs.cpu().numpy()[d], r["final_obs"][d], rtol=1e-6, atol=1e-5)
    np.testing.assert_array_equal(env.counters.cpu().numpy()[2], np.full(N, T // 37))


def test_mixed_launch_equals_separate_launches(gpu, built_lib):
    """One heterogeneous launch (boat helpers + owners + parachute + car waves) produces
    exactly what the separate per-type launches produce (ragged sizes)."""
    from sacenv import VecBoatEnv
    from sacenv.toys import MixedBatch
    cfg = {"base_settings": {"experiment": 6, "test_mode": 0}}
    b1 = VecBoatEnv(cfg, 3000, seed=5, device="cuda", max_episode_steps=13, n_helpers=16)
    b2 = VecBoatEnv(cfg, 3000, seed=5, device="cuda", max_episode_steps=13, n_helpers=16)
    p1, p2 = _toy_env(1, 1000, max_episode_steps=29), _toy_env(1, 1000, max_episode_steps=29)
    c1, c2 = _toy_env(2, 777, max_episode_steps=31), _toy_env(2, 777, max_episode_steps=31)
    mix = MixedBatch(b1, [p1, c1])
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    for k in range(60):
        a = torch.rand(3000, generator=g, device="cuda") * 2 - 1
        mix.step_async(a)
        b2.step_async(a)
        p2.step_async()
        c2.step_async()
    torch.cuda.synchronize()
    for x, y in ((b1, b2), (p1, p2), (c1, c2)):
        assert torch.equal(x.record, y.record)
        assert torch.equal(x.arena, y.arena)


@pytest.mark.parametrize("K", [1, 37, 128])
def test_mixed_segment_equals_mixed_steps(K, gpu, built_lib):
    """sacenv_mixed_segment (the mixed batch as ONE persistent launch of K steps) =
    K sacenv_mixed_step launches, bit for bit: boat and toy arenas (state, counters,
    the last record, terminal obs), with restarts and truncations inside the
    segments and refills between them (ragged sizes)."""
    from sacenv import VecBoatEnv
    from sacenv.toys import MixedBatch
    cfg = {"base_settings": {"experiment": 6, "test_mode": 0}}
    kw = dict(seed=5, device="cuda", max_episode_steps=23, n_helpers=16, auto_refill=False)
    b1, b2 = VecBoatEnv(cfg, 3000, **kw), VecBoatEnv(cfg, 3000, **kw)
    p1, p2 = _toy_env(1, 1000, max_episode_steps=29), _toy_env(1, 1000, max_episode_steps=29)
    c1, c2 = _toy_env(2, 777, max_episode_steps=31), _toy_env(2, 777, max_episode_steps=31)
    b1.reset()
    b2.reset()
    m1, m2 = MixedBatch(b1, [p1, c1]), MixedBatch(b2, [p2, c2])
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    acts = torch.rand((3 * K, 3000), generator=g, device="cuda") * 2 - 1
    for s in range(3):
        m1.segment_async(acts[s * K: (s + 1) * K], K)
        for k in range(s * K, (s + 1) * K):
            m2.step_async(acts[k])
        b1.refill()
        b2.refill()
        torch.cuda.synchronize()
        for name, x, y in (("boat", b1, b2), ("parachute", p1, p2), ("car", c1, c2)):
            assert torch.equal(x.arena, y.arena), (name, s)
    b1.check_status()
    if 3 * K > 31:   # the truncations (29 / 31 steps) fell inside the segments
        assert int(p1.counters.sum()) > 0 and int(c1.counters.sum()) > 0


def test_c5_mixed_segments_32768_each_vs_oracles(gpu, built_lib):
    """BASELINE configs[4] on the persistent mixed launch (the bench's --mixed path):
    128-step segments of boat exp 6 + parachute + car, 32 768 each; after every
    segment all six carried boat fields of a subsample vs the boat oracle stepped
    through the same 128 steps, every toy env's state and last obs vs the toy oracle."""
    from sacenv import VecBoatEnv
    from sacenv.toys import MixedBatch
    from toy_oracle import OracleToy
    N, SEGS, K = 32768, 3, 128
    rng = np.random.default_rng(4)
    seeds = np.arange(N, dtype=np.uint64) + 500
    boat = VecBoatEnv({"base_settings": {"experiment": 6, "test_mode": 0}}, N, seeds=seeds, device=gpu,
                      max_episode_steps=120, auto_refill=False)
    par, car = _toy_env(1, N, max_episode_steps=110), _toy_env(2, N, max_episode_steps=130)
    mix = MixedBatch(boat, [par, car])
    boat.reset()
    pick = np.sort(rng.choice(N, 192, replace=False))
    ora = OracleVecBoat(OracleConfig(experiment=6), seeds[pick], max_episode_steps=120)
    ora.reset()
    toys = [OracleToy(1, N, max_episode_steps=110), OracleToy(2, N, max_episode_steps=130)]
    ended = 0
    for s in range(SEGS):
        a = rng.uniform(-1, 1, (K, N)).astype(np.float32)
        mix.segment_async(torch.from_numpy(a).to(gpu), K)
        boat.refill()
        for k in range(K):
            ro = ora.step(a[k, pick])
            ended += int(ro["done"].sum())
            tr = [t.step() for t in toys]
        torch.cuda.synchronize()
        np.testing.assert_array_equal(boat.term.cpu().numpy()[pick], ro["term"], err_msg=f"segment {s}")
        np.testing.assert_allclose(boat.obs.cpu().numpy()[pick], ro["reset_obs"], rtol=OBS_TOL, atol=OBS_TOL)
        for f in ("s_x", "s_y", "s_r", "v_x", "v_y", "v_r"):
            err = np.abs(getattr(boat, f).cpu().numpy()[pick] - getattr(ora, f)).max()
            assert err <= STATE_TOL, (f, s, err)
        for env, r in ((par, tr[0]), (car, tr[1])):
            np.testing.assert_array_equal(env.term.cpu().numpy(), r["term"], err_msg=f"segment {s}")
            np.testing.assert_allclose(env.obs.cpu().numpy(), r["obs"], rtol=1e-6, atol=1e-5)
            np.testing.assert_allclose(env.state.cpu().numpy(), r["state"], rtol=0, atol=1e-5)
    np.testing.assert_array_equal(boat.counters.cpu().numpy().T[pick], ora.counters)
    boat.check_status()
    assert ended > 0


# ---------------------------------------------------------------- replay buffer (§8(f))

@pytest.mark.parametrize("case", ["partial", "wrapped", "one_row", "small"])
def test_replay_dropin_matches_reference_buffer(case, gpu, built_lib):
    """sacenv.replay.ReplayBuffer == agent.buffer.ReplayBuffer: same stored rows, same
    np.random.choice batches from numpy's global stream, same stream state after."""
    from sacenv.replay import ReplayBuffer
    z = golden("replay_buffer.npz")
    g = lambda k: z[f"{case}_{k}"]  # noqa: E731
    S, S2, A, R, D = g("S"), g("S2"), g("A"), g("R"), g("D")
    rb = ReplayBuffer(int(g("M")), (11,), 1, device="cuda")
    if len(R) <= 300:
        for i in range(len(R)):
            rb.store_transition(S[i], A[i], R[i], S2[i], bool(D[i]))
    else:  # batched store of the same sequence (ring wraps inside the call)
        rb._rb.store_batch(torch.from_numpy(S), torch.from_numpy(A), torch.from_numpy(R),
                           torch.from_numpy(S2), torch.from_numpy(D.astype(np.uint8)))
    assert rb.mem_cntr == len(R)
    np.random.seed(int(g("seed")))
    got = rb.sample_buffer(int(g("batch")))
    for x, k in zip(got, ("states", "actions", "rewards", "states_", "dones")):
        np.testing.assert_array_equal(x, g(k), err_msg=k)
    st = np.random.get_state()
    assert st[2] == int(g("pos_after"))
    np.testing.assert_array_equal(np.asarray(st[1], np.uint32), g("key_after"))


def test_replay_store_env_step_uses_final_obs(gpu, built_lib):
    """Batched path: transitions of a VecBoatEnv step; envs that auto-reset store their
    terminal obs as new_state; reference_terminal=False: terminal = this step reached
    the goal."""
    from sacenv import VecBoatEnv
    from sacenv.replay import DeviceReplayBuffer
    cfg = {"base_settings": {"experiment": 6, "test_mode": 1}, "boat_env": {"goal_line": 40}}
    env = VecBoatEnv(cfg, 512, seed=3, device="cuda", max_episode_steps=60, n_helpers=8)
    rb = DeviceReplayBuffer(50_000, (11,), 1, device="cuda", seed=5)
    obs = env.reset().clone()
    steps = 80
    a = torch.zeros(512, device="cuda")
    done_any = goal_any = False
    for k in range(steps):
        env.step(a)
        rb.store_env_step(obs, a.view(-1, 1), env, reference_terminal=False)
        d = env.done.bool()
        row0 = k * 512
        torch.cuda.synchronize()
        ns = rb.new_state_memory[row0: row0 + 512]
        assert torch.equal(ns[d], env.final_obs[d]) and torch.equal(ns[~d], env.obs[~d])
        assert torch.equal(rb.state_memory[row0: row0 + 512], obs)
        assert torch.equal(rb.terminal_memory[row0: row0 + 512].bool(), env.term == 1)
        assert torch.equal(rb.reward_memory[row0: row0 + 512], env.reward.double())
        done_any |= bool(d.any())
        goal_any |= bool((env.term == 1).any())
        obs = env.obs.clone()
    assert done_any and goal_any
    # sampling: indices follow np.random.choice on the buffer's own stream (seed 5)
    st, ac, rw, ns, tm, idx = rb.sample(1024)
    want = np.random.RandomState(5).choice(min(rb.mem_cntr, rb.mem_size), 1024)
    np.testing.assert_array_equal(idx.cpu().numpy(), want)
    assert torch.equal(st, rb.state_memory[idx]) and torch.equal(ns, rb.new_state_memory[idx])


def test_replay_store_with_host_count_equals_two_launch_store(gpu, built_lib):
    """sacenv_replay_store_env_at (the count from the host, one launch; what
    DeviceReplayBuffer.store_batch issues) leaves the arena -- rows, last_term bytes
    and the device mem_cntr -- exactly as sacenv_replay_store_env (device count, a
    second launch to advance it), across ring wraps and a call storing more rows
    than the ring holds."""
    from sacenv import _lib
    from sacenv.replay import DeviceReplayBuffer
    M = 1000
    a, b = (DeviceReplayBuffer(M, (11,), 1, device=gpu, seed=5) for _ in range(2))
    a.arena.zero_()            # (unwritten ring rows hold whatever the allocation held)
    b.arena.copy_(a.arena)
    lt_a, lt_b = (torch.zeros(2500, dtype=torch.uint8, device=gpu) for _ in range(2))
    g = torch.Generator(device=gpu).manual_seed(4)
    for n in (300, 300, 300, 300, 2500, 7, 650):
        st = torch.rand((n, 11), generator=g, device=gpu)
        ns = torch.rand((n, 11), generator=g, device=gpu)
        fo = torch.rand((n, 11), generator=g, device=gpu)
        ac = torch.rand((n, 1), generator=g, device=gpu)
        rw = torch.rand(n, generator=g, device=gpu, dtype=torch.float64)
        rw = rw.float() if a.params.reward_f32 else rw   # as store_batch hands it over
        cd = torch.randint(0, 7, (n,), generator=g, device=gpu, dtype=torch.uint8)
        a.store_batch(st, ac, rw, ns, cd, final_state=fo, last_term=lt_a[:n])
        _lib.check(b.lib.sacenv_replay_store_env(
            b._pp, b.arena.data_ptr(), n, st.data_ptr(), ac.data_ptr(), rw.data_ptr(), ns.data_ptr(),
            fo.data_ptr(), cd.data_ptr(), lt_b[:n].data_ptr(), b.stream))
        b.mem_cntr += n
        torch.cuda.synchronize()
        assert torch.equal(a.arena, b.arena) and torch.equal(lt_a, lt_b), n
        assert int(a._cntr.item()) == a.mem_cntr == b.mem_cntr == int(b._cntr.item())
    with pytest.raises((ValueError, _lib.SacenvError)):
        _lib.check(a.lib.sacenv_replay_store_env_at(a._pp, a.arena.data_ptr(), -1, 1, st.data_ptr(),
                                                    ac.data_ptr(), rw.data_ptr(), ns.data_ptr(), None,
                                                    cd.data_ptr(), None, a.stream))


def test_replay_store_env_step_reference_terminal_vs_main_loop(gpu, built_lib):
    """main.py:70-91 around the reference env + ReplayBuffer (main_loop_goal.npz): the
    device buffer holds the same rows, terminal following the env's persistent
    info['termination'] (sacenv_replay_store_env's last_term byte per env)."""
    from sacenv import VecBoatEnv
    from sacenv.replay import DeviceReplayBuffer
    z = golden("main_loop_goal.npz")
    E, S = z["term"].shape
    env = VecBoatEnv(_cfg_dict(z), E, seeds=z["seeds"], device=gpu, autoreset=True, n_helpers=8)
    rb = DeviceReplayBuffer(E * S, (11,), 1, device=gpu, seed=1)
    obs = env.reset().clone()
    acts = torch.from_numpy(np.ascontiguousarray(z["actions"].T)).to(gpu)
    for k in range(S):
        env.step(acts[k])
        rb.store_env_step(obs, acts[k].view(-1, 1), env)
        obs = env.obs.clone()
    torch.cuda.synchronize()
    assert rb.mem_cntr == E * S
    view = lambda t: t.cpu().numpy().reshape(S, E, *t.shape[1:]).swapaxes(0, 1)  # noqa: E731
    np.testing.assert_array_equal(view(rb.terminal_memory).astype(bool), z["terminal"])
    np.testing.assert_allclose(view(rb.state_memory), z["state"], rtol=0, atol=OBS_TOL)
    np.testing.assert_allclose(view(rb.new_state_memory), z["new_state"], rtol=0, atol=OBS_TOL)
    np.testing.assert_array_equal(view(rb.action_memory), z["action"])
    # the batched path stores the f32 reward the step writes (rewards reach ~1000)
    np.testing.assert_allclose(view(rb.reward_memory), z["reward"], rtol=1e-6, atol=STATE_TOL)


# ---------------------------------------------------------------- done compaction + device-list reset

@pytest.mark.parametrize("n,offset", [(0, 0), (1, 0), (63, 0), (4096, 0), (65537, 0), (70000, 3)])
def test_compact_done_matches_nonzero(n, offset, gpu, built_lib):
    from sacenv import _lib
    lib = _lib.load()
    g = torch.Generator(device="cuda")
    g.manual_seed(n + offset)
    buf = (torch.rand(n + offset + 1, generator=g, device="cuda") < 0.1).to(torch.uint8)
    buf[offset: offset + n: 97] = 7                       # nonzero values other than 1
    d = buf[offset: offset + n]                            # offset 3: unaligned start
    ids = torch.full((max(n, 1),), -1, dtype=torch.int32, device="cuda")
    cnt = torch.empty(1, dtype=torch.int32, device="cuda")
    _lib.check(lib.sacenv_compact_done(d.data_ptr(), n, ids.data_ptr(), cnt.data_ptr(),
                                       torch.cuda.current_stream().cuda_stream))
    want = torch.nonzero(d).flatten().to(torch.int32)
    assert int(cnt.item()) == want.numel()
    assert torch.equal(ids[: want.numel()], want)


@pytest.mark.parametrize("autoreset", [False, True])
def test_reset_done_equals_reset_of_ids(autoreset, gpu, built_lib):
    """reset_done (device compaction + device-count reset) == reset(ids) from the host."""
    from sacenv import VecBoatEnv
    cfg = {"base_settings": {"experiment": 6, "test_mode": 0}}
    kw = dict(seed=9, device="cuda", autoreset=autoreset, max_episode_steps=0, n_helpers=8)
    e1, e2 = VecBoatEnv(cfg, 3001, **kw), VecBoatEnv(cfg, 3001, **kw)
    g = torch.Generator(device="cuda")
    g.manual_seed(1)
    for k in range(40):
        a = torch.rand(3001, generator=g, device="cuda") * 2 - 1
        e1.step(a)
        e2.step(a)
        if k % 7 == 6:
            mask = (torch.rand(3001, generator=g, device="cuda") < 0.2).to(torch.uint8)
            e1.reset_done(mask)
            e2.reset(torch.nonzero(mask).flatten())
    torch.cuda.synchronize()
    assert torch.equal(e1.arena, e2.arena)


@pytest.mark.parametrize("dt,t_max", [(0.1, 30.0), (0.25, 12.0)])
def test_time_accumulation_carried_and_derived(dt, t_max, gpu, built_lib):
    """dt = 0.1 keeps t in HBM (t += dt rounds); dt = 0.25 derives t = index * dt (exact).
    Both must time out on the same step as the oracle's accumulated t (boat_env.py:69, :99)."""
    from sacenv import VecBoatEnv
    from sacenv.config import t_from_index
    assert t_from_index(0.25) and not t_from_index(0.1)
    N = 200
    seeds = np.arange(N, dtype=np.uint64) + 77
    cfg = {"base_settings": {"experiment": 6, "test_mode": 1, "dt": dt, "t_max": t_max}}
    env = VecBoatEnv(cfg, N, seeds=seeds, device=gpu, autoreset=True, n_helpers=8)
    ora = OracleVecBoat(OracleConfig(experiment=6, test_mode=1, dt=dt, t_max=t_max), seeds)
    env.reset()
    ora.reset()
    steps = int(round(t_max / dt)) + 5
    zero = np.zeros(N, np.float32)
    for k in range(steps):
        _, _, _, info = env.step(torch.zeros(N, device=gpu))
        r = ora.step(zero)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(info["term"].cpu().numpy(), r["term"], err_msg=f"step {k}")
        np.testing.assert_array_equal(env.t.cpu().numpy(), ora.t, err_msg=f"step {k}")
    assert (env.counters.cpu().numpy()[4] >= 1).all()   # every env timed out at least once


@pytest.mark.parametrize("exp", [1, 2, 3, 4, 5, 6])
def test_autoreset_all_experiments_ragged_vs_oracle(exp, gpu, built_lib):
    """Every experiment, a ragged env count (1000 = 15 full waves + 40), auto-reset with
    truncation and natural terminations (narrow track), all envs against the oracle:
    term codes bit-exact, obs / final_obs / final episode reward / state within tolerance."""
    from sacenv import VecBoatEnv
    N, S, TR = 1000, 160, 37
    seeds = (np.arange(N, dtype=np.uint64) * 7919 + 13) % (2 ** 32)
    cfg = {"base_settings": {"experiment": exp, "test_mode": 0}, "boat_env": {"track_width": 30}}
    env = VecBoatEnv(cfg, N, seeds=seeds, device=gpu, autoreset=True, max_episode_steps=TR,
                     n_helpers=9)
    ora = OracleVecBoat(OracleConfig(experiment=exp, test_mode=0, track_width=30), seeds,
                        max_episode_steps=TR)
    np.testing.assert_allclose(env.reset().cpu().numpy(), ora.reset(), rtol=OBS_TOL, atol=OBS_TOL)
    rng = np.random.default_rng(exp)
    n_nat = 0
    for k in range(S):
        a = rng.uniform(-1, 1, N).astype(np.float32)
        o, r, d, info = env.step(torch.from_numpy(a).to(gpu))
        ro = ora.step(a)
        torch.cuda.synchronize()
        term = info["term"].cpu().numpy()
        np.testing.assert_array_equal(term, ro["term"], err_msg=f"step {k}")
        done = term != 0
        n_nat += int(((term > 0) & (term < 6)).sum())
        np.testing.assert_allclose(o.cpu().numpy(), ro["reset_obs"], rtol=OBS_TOL, atol=OBS_TOL)
        np.testing.assert_allclose(r.cpu().numpy(), ro["reward"], rtol=1e-6, atol=1e-5)
        if done.any():
            np.testing.assert_allclose(info["final_obs"].cpu().numpy()[done], ro["obs"][done],
                                       rtol=OBS_TOL, atol=OBS_TOL)
            np.testing.assert_allclose(info["final_ep_reward"].cpu().numpy()[done],
                                       ro["ep_reward"][done], rtol=0, atol=1e-5)
        assert np.abs(env.s_x.cpu().numpy() - ora.s_x).max() <= STATE_TOL
        assert np.abs(env.s_y.cpu().numpy() - ora.s_y).max() <= STATE_TOL
    assert n_nat > 0
    np.testing.assert_array_equal(env.counters.cpu().numpy().T, ora.counters)


@pytest.mark.parametrize("exp", [4, 5, 6])
@pytest.mark.parametrize("autoreset", [False, True])
def test_wind_piece_cache_across_intervals_and_episodes(exp, autoreset, gpu, built_lib):
    """The step evaluates its wind from a per-env copy of its spline piece (layout.wind_coef),
    refreshed from the episode's slot only on a new episode or an interval crossing.
    Short wind tables (L = 120, 17 steps per knot interval) and frozen rudders (episodes
    run to the timeout, so every interval and the end-of-table clamp are crossed), for
    2.6 episodes: the wind each step uses equals the oracle's (wind.py:20-24, :69-99)."""
    from sacenv import VecBoatEnv
    N, t_max = 333, 30.0
    L = int(t_max / 0.25)
    seeds = np.arange(N, dtype=np.uint64) * 31 + 5
    cfg = {"base_settings": {"experiment": exp, "test_mode": 1, "t_max": t_max}}
    env = VecBoatEnv(cfg, N, seeds=seeds, device=gpu, autoreset=autoreset, n_helpers=8)
    ora = OracleVecBoat(OracleConfig(experiment=exp, test_mode=1, t_max=t_max), seeds)
    env.reset()
    ora.reset()
    zero = np.zeros(N, np.float32)
    crossed = 0
    for k in range(int(2.6 * L)):
        idx = torch.clamp(env.index, max=L - 1)
        wv, wa = env.wind_eval(torch.arange(N, device=gpu), idx)   # the wind this step will use
        wnext = torch.stack([wv, wa], 1).cpu().numpy()
        _, _, _, info = env.step(torch.zeros(N, device=gpu))
        r = ora.step(zero)
        torch.cuda.synchronize()
        np.testing.assert_allclose(wnext, r["wind"], rtol=0, atol=1e-12, err_msg=f"step {k}")
        term = info["term"].cpu().numpy()
        np.testing.assert_array_equal(term, r["term"], err_msg=f"step {k}")
        ended = np.flatnonzero(term)
        if ended.size and not autoreset:
            env.reset(ended)
        assert np.abs(env.s_y.cpu().numpy() - ora.s_y).max() <= STATE_TOL
        crossed += int((r["state"]["index"] % 17 == 0).sum())
    assert (env.counters.cpu().numpy()[4] >= 1).all()       # every env timed out
    assert crossed > 0


@pytest.mark.parametrize("exp,tmax,dt", [(6, 2500.0, 0.25), (4, 20.0, 0.25), (2, 2500.0, 0.25),
                                         (3, 2500.0, 0.25), (6, 20.0, 0.1)])
def test_rollout_equals_sequential_steps(exp, tmax, dt, gpu, built_lib):
    """sacenv_boat_rollout (K steps in one launch, state in registers) gives the records,
    terminal obs, counters and final state of K step() calls bit for bit, through
    auto-resets, wind-interval crossings (t_max 20: 11 steps per knot interval) and
    timeouts; then keeps matching across a refill. Covers every step-kernel instantiation:
    2, 1 and 0 wind curves, t from the index (dt 0.25) and t carried (dt 0.1)."""
    from sacenv import VecBoatEnv
    N, K = 777, 40
    cfg = {"base_settings": {"experiment": exp, "test_mode": 0, "t_max": tmax, "dt": dt},
           "boat_env": {"track_width": 30}}
    kw = dict(seed=11, device=gpu, autoreset=True, max_episode_steps=23, n_helpers=64)
    a_env, b_env = VecBoatEnv(cfg, N, **kw), VecBoatEnv(cfg, N, **kw)
    g = torch.Generator(device=gpu)
    g.manual_seed(exp)
    for rep in range(5):   # 200 steps: crosses a refill (period 128)
        acts = torch.rand((K, N), generator=g, device=gpu) * 2 - 1
        acts[:, ::7] *= 12.0   # some rudders break at once
        fin = torch.zeros((K, a_env.n_pad, 11), dtype=torch.float32, device=gpu)
        recs, _ = a_env.rollout(acts, final_obs=fin)
        for k in range(K):
            o, r, d, info = b_env.step(acts[k])
            ro, rr, rd, rt = a_env.record_views(recs[k])
            torch.testing.assert_close(ro, o, rtol=0, atol=0)
            torch.testing.assert_close(rr, r, rtol=0, atol=0)
            assert torch.equal(rd, d) and torch.equal(rt, info["term"]), (rep, k)
            done = d.bool()
            if done.any():
                torch.testing.assert_close(fin[k, :N][done], info["final_obs"][done], rtol=0, atol=0)
        names = ("s_x", "s_y", "s_r", "v_x", "v_y", "v_r", "rudder", "ep_reward", "index", "cons")
        for name in names + (("t",) if dt == 0.1 else ()):
            assert torch.equal(getattr(a_env, name), getattr(b_env, name)), (rep, name)
        assert torch.equal(a_env.counters, b_env.counters)
    a_env.check_status()
    b_env.check_status()


# ---------------------------------------------------------------- recorder (§8(f) rank 3)

def test_vec_recorder_reproduces_reference_episode_csv(tmp_path, gpu, built_lib):
    """VecRecorder on the reference's recorded exp-6 episode (wind table + start y replayed):
    the episode CSV matches the reference's own episode_0_data.csv row for row (state within
    1e-5, action and n exact), info.csv holds the reached_goal row and the episode reward."""
    import csv
    from sacenv import VecBoatEnv
    from sacenv.recorder import COLUMNS, VecRecorder
    z = golden("recorded_exp6.npz")
    tr, cols = z["trace"], [str(c) for c in z["columns"]]
    assert tuple(cols) == COLUMNS
    table = np.stack([z["wind_velocity"], z["wind_angle"]])
    env = VecBoatEnv({"base_settings": {"experiment": 6, "test_mode": 1}}, 3, device=gpu,
                     autoreset=False, wind_table=table, record_reward64=True)
    y0 = int(tr[0, cols.index("boat_position_y")])
    env.reset_explicit([0, 1, 2], [y0, y0, y0])
    rec = VecRecorder(env, [1], str(tmp_path), flush_steps=700)
    n = len(tr)
    acts = np.zeros(n, np.float32)
    acts[: n - 1] = tr[1:, cols.index("action_rudder")]       # row k+1 holds step k's action
    for k in range(n):
        rec.record()
        a = torch.full((3,), float(acts[k]), dtype=torch.float32, device=gpu)
        env.step(a)
        rec.after_step(a)
    rec.close()
    d = tmp_path / "episodes" / "env_1"
    with open(d / "episode_0_data.csv") as f:
        rows = list(csv.reader(f, delimiter=";"))
    assert tuple(rows[0]) == COLUMNS and len(rows) == n + 1
    got = np.array([[float(x) for x in r] for r in rows[1:]])
    state_cols = [cols.index(c) for c in COLUMNS[:5]] + [cols.index("rudder_angle")]
    np.testing.assert_allclose(got[:, state_cols], tr[:, state_cols], rtol=0, atol=1e-5)
    np.testing.assert_array_equal(got[:, cols.index("action_rudder")].astype(np.float32),
                                  tr[:, cols.index("action_rudder")].astype(np.float32))
    np.testing.assert_allclose(got[:, cols.index("reward")], tr[:, cols.index("reward")], rtol=1e-9, atol=1e-12)
    assert (got[:, cols.index("n")] == 20).all()
    with open(d / "info.csv") as f:
        info = list(csv.reader(f, delimiter=";"))
    assert info[0][0] == "termination" and info[1][0] == "reached_goal" and info[1][1] == "1"
    assert abs(float(info[1][-1]) - float(z["episode_reward"])) < 1e-6
    with open(d / "wind.csv") as f:
        w = np.array([[float(x) for x in r] for r in list(csv.reader(f, delimiter=";"))[1:]])
    np.testing.assert_array_equal(w, table.T)


@pytest.mark.parametrize("agent", ["native", "torch"])
def test_vec_sac_training_loop_runs_on_device(gpu, built_lib, agent):
    """§8(f) ranks 2 and 4: batched act + step + replay + SAC update (examples/train_vec_sac.py)."""
    import importlib.util
    import os
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                        "examples", "train_vec_sac.py")
    spec = importlib.util.spec_from_file_location("train_vec_sac", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    out = mod.main(["--envs", "2048", "--iters", "20", "--agent", agent])
    assert out["env_steps_per_s"] > 0 and out["losses"] is not None
    assert all(np.isfinite(out["losses"]))


# ---------------------------------------------------------------- configs at their stated sizes

def _subsample_run(env_factory, cfg, N, S, max_steps, pick, seed_base, act_seed):
    """Step a VecBoatEnv of N envs S steps with U(-1,1) actions; check the picked envs
    against the oracle run on just their seeds (term bit-exact, obs/state to tolerance)."""
    rng = np.random.default_rng(act_seed)
    seeds = np.arange(N, dtype=np.uint64) + seed_base
    env = env_factory(seeds)
    env.reset()
    ora = OracleVecBoat(cfg, seeds[pick], max_episode_steps=max_steps)
    ora.reset()
    ended = trunc = 0
    for k in range(S):
        a = rng.uniform(-1, 1, N).astype(np.float32)
        o, r, d, info = env.step(torch.from_numpy(a).to(env.device))
        ro = ora.step(a[pick])
        torch.cuda.synchronize()
        term = info["term"].cpu().numpy()[pick]
        np.testing.assert_array_equal(term, ro["term"], err_msg=f"step {k}")
        np.testing.assert_allclose(o.cpu().numpy()[pick], ro["reset_obs"], rtol=OBS_TOL, atol=OBS_TOL)
        dd = ro["done"].astype(bool)
        if dd.any():
            np.testing.assert_allclose(info["final_obs"].cpu().numpy()[pick][dd], ro["obs"][dd],
                                       rtol=OBS_TOL, atol=OBS_TOL)
        for f in ("s_x", "s_y", "v_x", "v_y", "s_r"):
            assert np.abs(getattr(env, f).cpu().numpy()[pick] - getattr(ora, f)).max() <= STATE_TOL, f
        ended += int(dd.sum())
        trunc += int((term == 6).sum())
    return ended, trunc


def test_c2_exp1_4096_envs_500_step_episodes(gpu, built_lib):
    """BASELINE configs[1] at its size: exp 1, 4 096 envs, episodes
    truncated at 500 steps, auto-reset; 256 envs checked against the oracle over 620
    steps (early endings and the step-500 truncation)."""
    from sacenv import VecBoatEnv
    N = 4096
    pick = np.sort(np.random.default_rng(2).choice(N, 256, replace=False))
    mk = lambda seeds: VecBoatEnv({"base_settings": {"experiment": 1, "test_mode": 0}}, N,  # noqa: E731
                                  seeds=seeds, device=gpu, max_episode_steps=500)
    ended, trunc = _subsample_run(mk, OracleConfig(experiment=1), N, 620, 500, pick, 77, 5)
    assert trunc > 0 and ended > trunc


def test_envs_beyond_130k_per_gpu(gpu, built_lib):
    """131 072 envs on one GPU (round 1 capped n_pad at 130 048 by 32-bit slot-ring
    offsets): the last owner waves, past the old cap, match the oracle."""
    from sacenv import VecBoatEnv
    N = 131072
    rng = np.random.default_rng(3)
    pick = np.sort(np.concatenate([rng.choice(130048, 64, replace=False), np.arange(N - 64, N)]))
    mk = lambda seeds: VecBoatEnv({"base_settings": {"experiment": 6, "test_mode": 0}}, N,  # noqa: E731
                                  seeds=seeds, device=gpu, max_episode_steps=30)
    ended, _ = _subsample_run(mk, OracleConfig(experiment=6), N, 70, 30, pick, 9, 6)
    assert ended >= 128


def test_c5_mixed_32768_each_vs_oracles(gpu, built_lib):
    """BASELINE configs[4] at its size: boat exp 6 + parachute + car, 32 768 envs each,
    ONE launch per step; a boat subsample vs the boat oracle, every toy env vs the toy
    oracle (auto-reset + truncation)."""
    from sacenv import VecBoatEnv
    from sacenv.toys import MixedBatch
    from toy_oracle import OracleToy
    N, S = 32768, 260
    rng = np.random.default_rng(4)
    seeds = np.arange(N, dtype=np.uint64) + 500
    boat = VecBoatEnv({"base_settings": {"experiment": 6, "test_mode": 0}}, N, seeds=seeds, device=gpu,
                      max_episode_steps=120)
    par, car = _toy_env(1, N, max_episode_steps=110), _toy_env(2, N, max_episode_steps=130)
    mix = MixedBatch(boat, [par, car])
    boat.reset()
    pick = np.sort(rng.choice(N, 192, replace=False))
    ora = OracleVecBoat(OracleConfig(experiment=6), seeds[pick], max_episode_steps=120)
    ora.reset()
    toys = [OracleToy(1, N, max_episode_steps=110), OracleToy(2, N, max_episode_steps=130)]
    for k in range(S):
        a = rng.uniform(-1, 1, N).astype(np.float32)
        mix.step_async(torch.from_numpy(a).to(gpu))
        ro = ora.step(a[pick])
        tr = [t.step() for t in toys]
        torch.cuda.synchronize()
        np.testing.assert_array_equal(boat.term.cpu().numpy()[pick], ro["term"], err_msg=f"step {k}")
        np.testing.assert_allclose(boat.obs.cpu().numpy()[pick], ro["reset_obs"], rtol=OBS_TOL, atol=OBS_TOL)
        for f in ("s_x", "s_y", "s_r", "v_x", "v_y", "v_r"):   # every carried field
            err = np.abs(getattr(boat, f).cpu().numpy()[pick] - getattr(ora, f)).max()
            assert err <= STATE_TOL, (f, k, err)
        for env, r in ((par, tr[0]), (car, tr[1])):
            np.testing.assert_array_equal(env.term.cpu().numpy(), r["term"], err_msg=f"step {k}")
            np.testing.assert_allclose(env.obs.cpu().numpy(), r["obs"], rtol=1e-6, atol=1e-5)
            np.testing.assert_allclose(env.state.cpu().numpy(), r["state"], rtol=0, atol=1e-5)
    assert boat.counters.cpu().numpy().sum() > 0


# ---------------------------------------------------------------- pooled transition rows (§8(e))

@pytest.mark.parametrize("exp", [2, 6])
def test_step_pooled_row_equals_step_outputs(exp, gpu, built_lib):
    """sacenv_boat_step_pooled = sacenv_boat_step (arena bit-identical) + the 53-B
    transition row: s' = the pre-reset obs (final_obs where done), reward, action,
    term, obs3_next = the new episode's obs[3] (experiment 2); TransitionStream
    rebuilds each next s (the returned obs) bit-exactly from consecutive rows."""
    from sacenv import VecBoatEnv, _lib
    from sacenv.dist import TransitionLayout, TransitionStream
    cfg = {"base_settings": {"experiment": exp, "test_mode": 0}, "boat_env": {"track_width": 30}}
    N = 3000
    a_env = VecBoatEnv(cfg, N, seed=11, device=gpu, max_episode_steps=40, n_helpers=64)
    b_env = VecBoatEnv(cfg, N, seed=11, device=gpu, max_episode_steps=40, n_helpers=64)
    a_env.reset()
    obs0 = b_env.reset().clone()
    lay = TransitionLayout(N, b_env.n_pad, exp)
    row = torch.empty(lay.nbytes, dtype=torch.uint8, device=gpu)
    stream = TransitionStream(lay, 1, obs0, b_env.first_obs_template())
    assert lay.nbytes == (57 if exp == 2 else 53) * b_env.n_pad
    g = torch.Generator(device=gpu)
    g.manual_seed(5)
    ended = 0
    for k in range(150):
        act = torch.rand(N, generator=g, device=gpu) * 2 - 1
        a_env.step_async(act)
        b_env.step_pooled_async(act, row)
        torch.cuda.synchronize()
        assert torch.equal(a_env.arena, b_env.arena), f"step {k}"
        sp, rew, ac, term, obs3 = lay.views(row)
        d = a_env.done.bool()
        assert torch.equal(term != 0, d) and torch.equal(term, a_env.term)
        assert torch.equal(rew, a_env.reward) and torch.equal(ac, act)
        assert torch.equal(sp[d], a_env.final_obs[d]) and torch.equal(sp[~d], a_env.obs[~d])
        if exp == 2:
            assert torch.equal(obs3[d], a_env.obs[d][:, 3])
        else:
            assert obs3 is None
        s, a2, r2, sn, code = stream.push(row)
        assert torch.equal(sn[d], a_env.final_obs[d]) and torch.equal(sn[~d], a_env.obs[~d]), f"step {k}: s'"
        assert torch.equal(stream.prev, a_env.obs), f"step {k}: rebuilt next s"
        ended += int(d.sum())
    assert ended > 1000


def test_mixed_step_pooled_boat_row(gpu, built_lib):
    """The mixed launch writes the same boat transition row as the boat's own pooled step."""
    from sacenv import VecBoatEnv, _lib
    from sacenv.toys import MixedBatch
    cfg = {"base_settings": {"experiment": 6, "test_mode": 0}}
    b1 = VecBoatEnv(cfg, 1000, seed=2, device=gpu, max_episode_steps=17, n_helpers=16)
    b2 = VecBoatEnv(cfg, 1000, seed=2, device=gpu, max_episode_steps=17, n_helpers=16)
    mix = MixedBatch(b1, [_toy_env(1, 500, max_episode_steps=9)])
    r1 = torch.empty(_lib.TRANS_BYTES * b1.n_pad, dtype=torch.uint8, device=gpu)
    r2 = torch.empty_like(r1)
    g = torch.Generator(device=gpu)
    g.manual_seed(1)
    for k in range(40):
        a = torch.rand(1000, generator=g, device=gpu) * 2 - 1
        mix.step_async(a, r1)
        b2.step_pooled_async(a, r2)
        torch.cuda.synchronize()
        assert torch.equal(r1, r2), f"step {k}"
    with pytest.raises(ValueError):
        b2.step_pooled_async(a, r2[:-16])
