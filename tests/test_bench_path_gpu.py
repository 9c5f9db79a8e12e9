"""The bench's exact timed path under parity.

``bench.py`` times 256-step segments of the BASELINE config (exp 6, 65 536
envs, 500-step episodes, in-kernel auto-reset, the default refill helpers (12 288),
``auto_refill=False`` with the refill placed after every segment), each one
persistent ``sacenv_boat_segment`` launch (the default ``--launch segment``) or
one hipGraph replay of 256 ``k_step`` launches (``--launch step``). This test
builds that workload with bench's own ``make_workload`` and drives it with
bench's own ``SegmentRunner`` -- ``prepare()`` (warm-up, capture, the first
pass over the action table) and five timed-path segments -- in both modes,
next to an eager twin (``--no-graph``: the same runner issuing the same steps
as separate launches), and checks:

(a) after ``prepare()`` and after every segment (each followed by its refill),
    the three arenas -- carried state, slot rings, MT19937 states, counters, the
    last record and terminal obs -- are bit-identical;
(b) every step of the eager twin against ``OracleVecBoat`` on a 256-env
    subsample: termination codes bit-exact, obs and terminal obs within
    OBS_TOL, the six carried state fields (s_x, s_y, s_r, v_x, v_y, v_r) within
    STATE_TOL (BASELINE north_star: 1e-5), rewards and episode rewards; the
    cumulative info counters at the end.

Together: every step of the graph-replayed timed path matches the reference
restatement. The replayed segments must contain refills and step-500
truncations (asserted). Reference: environment/boat_env.py:67-126.
"""
import numpy as np
import pytest
import torch

from boat_oracle import OracleConfig, OracleVecBoat

pytestmark = pytest.mark.gpu

STATE_TOL = 1e-5
OBS_TOL = 1e-6
STATE = ("s_x", "s_y", "s_r", "v_x", "v_y", "v_r")
N_SEGMENTS = 5


def _picked(t, pick_d):
    return t.index_select(0, pick_d).cpu().numpy()


def _same(env, ref) -> bool:
    return torch.equal(env.arena, ref.arena)


def test_bench_timed_path_equals_eager_and_oracle(gpu, built_lib):
    import bench
    args_q = bench.parse(["--no-cpu-baseline"])
    args_g = bench.parse(["--no-cpu-baseline", "--launch", "step"])
    args_e = bench.parse(["--no-cpu-baseline", "--no-graph"])
    assert args_q.launch == "segment"   # the default the driver times
    assert (args_q.envs, args_q.experiment, args_q.episode_steps, args_q.helpers) == (65536, 6, 500, None)
    wls = [bench.make_workload(a, 0, gpu) for a in (args_q, args_g, args_e)]
    wl_e = wls[-1]
    envs = [w.envs[0] for w in wls]
    env_g, env_e = envs[1], envs[2]
    assert not env_g.auto_refill and env_g.autoreset
    torch.cuda.synchronize()
    for w, env in zip(wls, envs):
        assert torch.equal(w.actions, wl_e.actions) and _same(env, env_e)

    N = env_e.num_envs
    pick = np.sort(np.random.default_rng(7).choice(N, 256, replace=False))
    pick_d = torch.from_numpy(pick).to(gpu)
    ora = OracleVecBoat(OracleConfig(experiment=6), env_e.seeds[pick], max_episode_steps=500)
    ora.reset()
    acts = wl_e.actions.cpu().numpy()
    seen = {"steps": 0, "ended": 0, "trunc": 0, "phase": "prepare", "trunc_in_segments": 0}

    def on_step(k):
        """After eager step k (actions row k % 512): the subsample against the oracle."""
        ro = ora.step(acts[k % bench.ACTION_STEPS][pick])
        torch.cuda.synchronize()
        term = _picked(env_e.term, pick_d)
        np.testing.assert_array_equal(term, ro["term"], err_msg=f"step {seen['steps']}")
        np.testing.assert_array_equal(_picked(env_e.done, pick_d), ro["done"])
        np.testing.assert_allclose(_picked(env_e.obs, pick_d), ro["reset_obs"], rtol=OBS_TOL, atol=OBS_TOL)
        np.testing.assert_allclose(_picked(env_e.reward, pick_d), ro["reward"], rtol=1e-6, atol=1e-6)
        for f in STATE:
            err = np.abs(_picked(getattr(env_e, f), pick_d) - getattr(ora, f)).max()
            assert err <= STATE_TOL, (f, seen["steps"], err)
        d = ro["done"].astype(bool)
        if d.any():
            np.testing.assert_allclose(_picked(env_e.final_obs, pick_d)[d], ro["obs"][d], rtol=OBS_TOL,
                                       atol=OBS_TOL)
            np.testing.assert_allclose(_picked(env_e.final_ep_reward, pick_d)[d], ro["ep_reward"][d],
                                       rtol=0, atol=1e-4)
        seen["steps"] += 1
        seen["ended"] += int(d.sum())
        n_tr = int((term == 6).sum())
        seen["trunc"] += n_tr
        if seen["phase"] == "segments":
            seen["trunc_in_segments"] += n_tr

    runs = [bench.SegmentRunner(a, w, gpu) for a, w in zip((args_q, args_g, args_e), wls)]
    names = ("segment", "graph")
    assert [r.mode for r in runs] == ["segment", "graph", "eager"]
    for r in runs[:2]:
        r.prepare()
    runs[2].prepare(on_step=on_step)
    torch.cuda.synchronize()
    assert all(r.first_replays == 512 for r in runs)
    for name, env in zip(names, envs):
        assert _same(env, env_e), f"{name} arena differs after prepare()"

    seen["phase"] = "segments"
    refills0 = [int(env.status[0].item()) for env in envs]
    k = 0
    for s in range(N_SEGMENTS):
        ks = [r.segment(k) for r in runs[:2]]
        ke = runs[2].segment(k, on_step=on_step)
        assert ks == [ke] * 2 and ke == k + bench.SEG
        k = ke
        torch.cuda.synchronize()
        for name, env in zip(names, envs):
            if not _same(env, env_e):
                diff = torch.nonzero(env.arena != env_e.arena)[:8, 0].tolist()
                raise AssertionError(f"{name} arena differs after segment {s} at bytes {diff}")
            for f in STATE:  # the timed-path env itself, at the segment boundary
                assert np.abs(_picked(getattr(env, f), pick_d) - getattr(ora, f)).max() <= STATE_TOL, f
    for env in envs:
        env.check_status()
    for r0, env in zip(refills0, envs):
        assert int(env.status[0].item()) - r0 == N_SEGMENTS   # one refill per segment
    np.testing.assert_array_equal(_picked(env_g.counters.t().contiguous(), pick_d), ora.counters)
    assert seen["steps"] == 3 + 512 + N_SEGMENTS * bench.SEG
    assert seen["trunc_in_segments"] > 0 and seen["ended"] > 256, seen
