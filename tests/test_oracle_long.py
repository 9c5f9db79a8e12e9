"""Pin the CPU oracles to the reference's long scripted runs (tests/golden/long_*.npz).

``make_golden.py run_long`` drove the reference ``BoatEnv`` for 10 000 steps on default
configs with scripted rudder programs: spins to |s_r| ~ 240 rad,
a U-turn back across s_x = 0 inside the track, waypoint orbits that end in the
default-t_max timeout, and a slalom whose heading swings past -pi/2 and +pi/2 in one
episode. Each fixture records which reference branches it reached (``hits_*``); the
first test asserts them, so a regenerated fixture that lost a branch fails here.

Every step: term and done exact, the f64 reward. Kept steps (``keep``): the full state,
obs, wind, episode reward, and the reset draws of episodes that ended.
"""
import numpy as np
import pytest

from boat_oracle import OracleVecBoat, config_from_fixture
from conftest import golden, long_fixtures

STATE_TOL = 1e-9


def test_long_fixtures_reach_the_turnaround_branches():
    """boat_env.py:90 (s_x < 0 inside the track), :98-101 (t_max = 2500 default,
    10 000 steps), :107-108 (rudder penalty), :110-111 (heading penalty, both signs)."""
    tot = {k: 0 for k in ("heading_pos", "heading_neg", "rudder_penalty", "oob_sx_neg",
                          "timeout_default")}
    for name in long_fixtures():
        z = golden(name)
        assert int(z["n_steps"]) == 10000
        for k in tot:
            tot[k] += int(z[f"hits_{k}"])
        if "slalom" in name:   # one episode swinging past both signs
            assert int(z["hits_heading_pos"]) > 0 and int(z["hits_heading_neg"]) > 0
        else:                  # default track and t_max
            assert float(z["cfg_t_max"]) == 2500 and float(z["cfg_track_width"]) == 800
            assert float(z["hits_max_abs_s_r"]) > 200   # the spin: sincos far from [-pi, pi]
    assert all(v > 0 for v in tot.values()), tot
    # and the runs end the way the hits say
    z = golden("long_exp1.npz")
    assert (z["term"] == 5).sum() == 3 and (z["term"] == 2).sum() == 1


@pytest.mark.parametrize("name", long_fixtures())
def test_oracle_matches_reference_long(name):
    z = golden(name)
    o = OracleVecBoat(config_from_fixture(z), z["seeds"])
    np.testing.assert_allclose(o.reset(), z["init_obs"], rtol=0, atol=1e-15)
    np.testing.assert_array_equal(o.start_y, z["init_start_y"])
    keep = {int(k): j for j, k in enumerate(z["keep"])}
    fields = [str(f) for f in z["state_fields"]]
    E, S = z["reward"].shape
    worst = 0.0
    for k in range(S):
        r = o.step(z["actions"][:, k])
        np.testing.assert_array_equal(r["term"], z["term"][:, k], err_msg=f"step {k}")
        np.testing.assert_array_equal(r["done"], z["done"][:, k], err_msg=f"step {k}")
        np.testing.assert_allclose(r["reward"], z["reward"][:, k], rtol=0, atol=1e-9)
        j = keep.get(k)
        if j is None:
            continue
        st = np.stack([r["state"][f] for f in fields], 1)
        worst = max(worst, float(np.abs(st - z["state"][:, j]).max()))
        np.testing.assert_allclose(st, z["state"][:, j], rtol=0, atol=STATE_TOL, err_msg=f"step {k}")
        np.testing.assert_allclose(r["obs"], z["obs"][:, j], rtol=0, atol=1e-12)
        np.testing.assert_allclose(r["ep_reward"], z["ep_reward"][:, j], rtol=0, atol=1e-7)
        np.testing.assert_allclose(r["wind"], z["wind"][:, j], rtol=0, atol=1e-13)
        d = z["done"][:, k].astype(bool)
        if d.any():
            np.testing.assert_allclose(r["reset_obs"][d], z["reset_obs"][:, j][d], atol=1e-15)
            np.testing.assert_array_equal(o.start_y[d], z["start_y"][:, j][d])
    np.testing.assert_array_equal(o.counters, z["counters"])
    print(f"{name}: worst state err {worst:.3e}")


@pytest.mark.parametrize("name", long_fixtures())
def test_scalar_oracle_matches_reference_long(name):
    from boat_scalar import ScalarBoat
    z = golden(name)
    cfg = config_from_fixture(z)
    keep = {int(k): j for j, k in enumerate(z["keep"])}
    E, S = z["reward"].shape
    for e in range(E):
        b = ScalarBoat(cfg, int(z["seeds"][e]))
        b.reset()
        for k in range(S):
            obs, rew, term = b.step(float(z["actions"][e, k]))
            assert term == z["term"][e, k], (name, e, k)
            assert abs(rew - z["reward"][e, k]) <= 1e-9, (name, e, k)
            j = keep.get(k)
            if j is not None:
                st = (b.s_x, b.s_y, b.s_r, b.v_x, b.v_y, b.v_r, b.a_x, b.a_y, b.a_r, b.rudder, b.t,
                      b.fuel, b.index)
                np.testing.assert_allclose(st, z["state"][e, j], rtol=0, atol=STATE_TOL)
            if z["done"][e, k]:
                b.reset()
        np.testing.assert_array_equal(b.counters, z["counters"][e])
