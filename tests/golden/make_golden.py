"""Generate the golden fixtures under tests/golden/ from the reference itself.

Runs ONLY in the build container (needs /root/reference); the outputs are
plain ``.npz`` data committed next to this script. Nothing here is imported
by the product package, by smoke() or by bench.py.

Fixture kinds
-------------
``seeded_<name>.npz``
    The reference ``BoatEnv`` (``environment/boat_env.py:9-140``) driven the
    way ``main.py:70-91`` drives it: ``np.random.seed(seed)`` -> ``BoatEnv(cfg)``
    (constructor draws one ``Boat``, ``boat_env.py:15``) -> ``reset()`` -> ``step``
    with float32-valued actions, ``reset()`` again whenever ``done``.
    One independent reference env (one global-RNG seed) per fixture env.
``wind_exp<k>.npz``
    ``Wind`` tables (``wind.py:26-99``) for many seeds, sampled at fixed
    indices, plus each table's min/max (pins the spline and the min-max
    renormalisation, ``wind.py:87-89``).
``toy_parachute.npz`` / ``toy_car.npz``
    The reference toy scripts (``environment/toy_parachute.py``,
    ``environment/toy_car.py``) run as ``__main__`` with the ``Scope`` plot
    replaced by a capture of the recorded signals.
``replay_buffer.npz``
    The reference ``ReplayBuffer`` (``agent/buffer.py:3-35``): stored
    transitions, then ``sample_buffer`` under a seeded global numpy stream
    (batches and the RNG state after sampling), at several fill levels.
``main_loop_goal.npz``
    ``main.py:70-91``'s loop around the reference ``BoatEnv`` and ``ReplayBuffer``:
    the transitions it stores, with ``terminal = info['termination'] ==
    'reached_goal'`` (``main.py:83-88``). ``info['termination']`` persists
    across steps and resets (``boat_env.py:24-32,120-126``), so after a goal
    episode later steps are stored terminal until another ending overwrites it.
``sac_learn.npz``
    The reference ``ContinuousAgent`` (``agent/continuous_agent.py:9-154``, networks
    ``networks/networks.py:14-133``) built under ``torch.manual_seed(0)`` on the CPU,
    then ``learn()`` on fixed 1 024-row batches (``sample_buffer`` returns them) with
    the policy's ``Normal.sample``/``rsample`` drawing recorded standard normals
    (``loc + eps * scale``): the losses of each call and every network's weights
    after the calls.
``long_<name>.npz``
    ``run_long``: the reference ``BoatEnv`` under scripted rudder programs for 10 000
    steps on default configs (turns past +-pi/2, back across s_x = 0, the default
    t_max timeout, spins to hundreds of radians); the actions are recorded.
``recorded_exp<k>.npz``
    The reference's own recorded runs under
    ``ressources/settings_visualized/experiment_setting_<k>/`` converted from
    CSV (data files the reference ships).

Usage: ``python tests/golden/make_golden.py`` (writes into tests/golden/).
"""
from __future__ import annotations

import csv
import os
import tempfile
import types

import numpy as np

import _refharness as H

HERE = os.path.dirname(os.path.abspath(__file__))

# term codes: order of the info-dict keys, boat_env.py:24-32
TERM_CODES = {"": 0, "reached_goal": 1, "out_of_bounds": 2, "out_of_fuel": 3,
              "rudder_broken": 4, "timeout": 5}

STATE_FIELDS = ("s_x", "s_y", "s_r", "v_x", "v_y", "v_r", "a_x", "a_y", "a_r",
                "rudder_angle", "t", "fuel", "index")

SEEDS = np.array([0, 1, 7, 12345, 2**31 + 11, 2**32 - 1], dtype=np.uint64)


def _state(boat) -> list[float]:
    return [float(getattr(boat, f)) for f in STATE_FIELDS]


def run_seeded(name, overrides, n_steps, action_kind, seeds=SEEDS, action_seed=0):
    be = H.boat_env_module()
    cfg = H.load_config(overrides)
    E, S = len(seeds), n_steps
    rng = np.random.default_rng(action_seed)
    if action_kind == "uniform":
        actions = rng.uniform(-1.0, 1.0, size=(E, S)).astype(np.float32)
    elif action_kind == "zero":
        actions = np.zeros((E, S), np.float32)
    elif action_kind == "big":
        actions = rng.choice(np.array([-5.0, 5.0, 0.3], np.float32), size=(E, S))
    else:
        raise ValueError(action_kind)

    out = {k: [] for k in ("obs", "reward", "done", "term", "state", "ep_reward",
                           "wind", "reset_obs", "reset_state", "start_y",
                           "init_obs", "init_state", "init_start_y", "counters")}
    for e, seed in enumerate(seeds):
        np.random.seed(int(seed))
        env = be.BoatEnv(cfg, types.SimpleNamespace(experiment_dir=tempfile.mkdtemp()))
        # main.py:72 - reset before the first step
        obs0 = env.reset()
        out["init_obs"].append(np.asarray(obs0, np.float64))
        out["init_state"].append(_state(env.boat))
        out["init_start_y"].append(int(env.boat.s_y_start))
        rows = {k: [] for k in ("obs", "reward", "done", "term", "state", "ep_reward",
                                "wind", "reset_obs", "reset_state", "start_y")}
        for k in range(S):
            idx = env.boat.index
            wv, wa = env.boat.wind.get_wind(idx)
            a = np.array([float(actions[e, k])], dtype=np.float64)
            o, r, d, info = env.step(a)
            rows["wind"].append([float(wv), float(wa)])
            rows["obs"].append(np.asarray(o, np.float64))
            rows["reward"].append(float(r))
            rows["done"].append(bool(d))
            rows["term"].append(TERM_CODES[info["termination"]] if d else 0)
            rows["state"].append(_state(env.boat))
            rows["ep_reward"].append(float(info["episode_reward"]))
            if d:
                ro = env.reset()
                rows["reset_obs"].append(np.asarray(ro, np.float64))
                rows["reset_state"].append(_state(env.boat))
                rows["start_y"].append(int(env.boat.s_y_start))
            else:
                rows["reset_obs"].append(np.full(11, np.nan))
                rows["reset_state"].append([np.nan] * len(STATE_FIELDS))
                rows["start_y"].append(0)
        for kk, v in rows.items():
            out[kk].append(v)
        out["counters"].append([env.info[k] for k in
                                ("reached_goal", "out_of_bounds", "out_of_fuel",
                                 "rudder_broken", "timeout")])

    flat = {k: np.asarray(v) for k, v in out.items()}
    flat["obs"] = flat["obs"].astype(np.float64)
    flat["done"] = flat["done"].astype(np.uint8)
    flat["term"] = flat["term"].astype(np.uint8)
    flat["start_y"] = flat["start_y"].astype(np.int32)
    flat["seeds"] = np.asarray(seeds, np.uint64)
    flat["actions"] = actions
    flat["state_fields"] = np.array(STATE_FIELDS)
    cfg_vals = _cfg_vector(cfg)
    flat.update(cfg_vals)
    path = os.path.join(HERE, f"seeded_{name}.npz")
    np.savez_compressed(path, **flat)
    n_done = int(flat["done"].sum())
    print(f"{path}: E={E} S={S} episodes_ended={n_done} "
          f"terms={np.bincount(flat['term'].ravel(), minlength=6).tolist()}")


def _cfg_vector(cfg):
    """Config values the fixture was produced with (flat, for the tests)."""
    return {
        "cfg_experiment": np.int32(int(cfg.base_settings.experiment)),
        "cfg_test_mode": np.int32(int(cfg.base_settings.test_mode)),
        "cfg_dt": np.float64(cfg.base_settings.dt),
        "cfg_t_max": np.float64(cfg.base_settings.t_max),
        "cfg_fuel": np.int64(cfg.boat.fuel),
        "cfg_track_width": np.float64(cfg.boat_env.track_width),
        "cfg_goal_line": np.float64(cfg.boat_env.goal_line),
        "cfg_oob_offset": np.float64(cfg.boat_env.boat_out_of_bounds_offset),
    }


WIND_IDX = np.unique(np.concatenate([np.arange(0, 10000, 97), [9998, 9999]]))


def run_wind(exp, n_seeds=64, t_max=None):
    be = H.boat_env_module()
    over = {"base_settings": {"experiment": exp}}
    if t_max is not None:
        over["base_settings"]["t_max"] = t_max
    cfg = H.load_config(over)
    L = int(cfg.base_settings.t_max / cfg.base_settings.dt)
    idx = WIND_IDX[WIND_IDX < L] if t_max is None else np.arange(L)
    vel, ang, vmin, vmax, amin, amax, sy = [], [], [], [], [], [], []
    seeds = np.arange(1000, 1000 + n_seeds, dtype=np.uint64)
    for s in seeds:
        np.random.seed(int(s))
        boat = be.Boat(cfg)       # randint then Wind draws (boat_env.py:147-156)
        wv = np.asarray(boat.wind.wind_velocity, np.float64)
        wa = np.asarray(boat.wind.wind_angle, np.float64)
        vel.append(wv[idx]); ang.append(wa[idx])
        vmin.append(wv.min()); vmax.append(wv.max()); amin.append(wa.min()); amax.append(wa.max())
        sy.append(int(boat.s_y_start))
    suffix = "" if t_max is None else f"_tmax{t_max:g}"
    path = os.path.join(HERE, f"wind_exp{exp}{suffix}.npz")
    np.savez_compressed(path, seeds=seeds, idx=idx.astype(np.int32), L=np.int32(L),
                        vel=np.asarray(vel), ang=np.asarray(ang),
                        vmin=np.asarray(vmin), vmax=np.asarray(vmax),
                        amin=np.asarray(amin), amax=np.asarray(amax),
                        start_y=np.asarray(sy, np.int32),
                        experiment=np.int32(exp),
                        max_velocity=np.float64(cfg.wind.max_velocity),
                        direction=np.float64(cfg.wind.direction))
    print(f"{path}: seeds={n_seeds} L={L}")


def convert_recorded(exp):
    d = os.path.join(H.REF_ROOT, "ressources", "settings_visualized",
                     f"experiment_setting_{exp}")

    def read(p):
        with open(p) as f:
            rows = list(csv.reader(f, delimiter=";"))
        return rows[0], rows[1:]

    hdr, rows = read(os.path.join(d, "episodes", "episode_0_data.csv"))
    data = np.array([[float(x) for x in r] for r in rows], np.float64)
    whdr, wrows = read(os.path.join(d, "episodes", "wind.csv"))
    wind = np.array([[float(x) for x in r] for r in wrows], np.float64)
    thdr, trows = read(os.path.join(d, "terminations.csv"))
    term = dict(zip(thdr, trows[0]))
    path = os.path.join(HERE, f"recorded_exp{exp}.npz")
    np.savez_compressed(path, columns=np.array(hdr), trace=data,
                        wind_velocity=wind[:, 0], wind_angle=wind[:, 1],
                        termination=np.array(term["termination"]),
                        episode_reward=np.float64(term["episode_reward"]),
                        experiment=np.int32(exp))
    print(f"{path}: rows={len(data)} term={term['termination']}")


def run_toys():
    """toy_parachute.py:7-41 / toy_car.py:5-33 as scripts; capture Scope signals."""
    import runpy
    import sys
    H.install_standins()
    env_dir = os.path.join(H.REF_ROOT, "environment")
    if env_dir not in sys.path:
        sys.path.insert(0, env_dir)
    import control_theory.control_blocks as cb  # reference module
    captured = {}

    def capture(self, file_name="scope"):
        captured["signals"] = [list(map(float, s)) for s in self.signals]
        captured["labels"] = list(self.labels)

    orig = cb.Scope.create_time_scope
    cb.Scope.create_time_scope = capture
    try:
        for name in ("toy_parachute", "toy_car"):
            captured.clear()
            runpy.run_path(os.path.join(env_dir, f"{name}.py"), run_name="__main__")
            sig = np.array(captured["signals"], dtype=np.float64)
            path = os.path.join(HERE, f"{name}.npz")
            np.savez_compressed(path, signals=sig, labels=np.array(captured["labels"]))
            print(f"{path}: signals {sig.shape}")
    finally:
        cb.Scope.create_time_scope = orig


def run_replay():
    """agent/buffer.py ReplayBuffer: stores + np.random.choice sampling from the
    global stream, several fill levels (partial, wrapped, one row)."""
    H.install_standins()
    from agent.buffer import ReplayBuffer  # reference module
    cases = {"partial": (1000, 300, 64, 11), "wrapped": (1000, 2500, 1024, 12),
             "one_row": (50, 1, 16, 13), "small": (7, 5, 300, 14)}
    out = {}
    for name, (M, n_store, batch, seed) in cases.items():
        rng = np.random.default_rng(seed)
        rb = ReplayBuffer(M, (11,), 1)
        S = rng.standard_normal((n_store, 11)).astype(np.float32)
        S2 = rng.standard_normal((n_store, 11)).astype(np.float32)
        A = rng.uniform(-1, 1, (n_store, 1)).astype(np.float32)
        R = rng.standard_normal(n_store)
        Dn = rng.random(n_store) < 0.1
        for i in range(n_store):
            rb.store_transition(S[i], A[i], R[i], S2[i], bool(Dn[i]))
        np.random.seed(seed * 7 + 1)
        b = rb.sample_buffer(batch)
        after = np.random.get_state()
        out.update({f"{name}_{k}": v for k, v in dict(
            M=M, S=S, S2=S2, A=A, R=R, D=Dn, seed=seed * 7 + 1, batch=batch,
            states=b[0], actions=b[1], rewards=b[2], states_=b[3], dones=b[4],
            key_after=np.asarray(after[1], np.uint32), pos_after=after[2]).items()})
    path = os.path.join(HERE, "replay_buffer.npz")
    np.savez_compressed(path, cases=np.array(list(cases)), **out)
    print(f"{path}: {list(cases)}")


def run_main_loop(n_steps=700, seeds=SEEDS, action_seed=21):
    """main.py:70-91 with a reference ReplayBuffer: what the loop stores."""
    be = H.boat_env_module()
    from agent.buffer import ReplayBuffer  # reference module
    cfg = H.load_config({"base_settings": {"experiment": 6, "test_mode": 0},
                         "boat_env": {"goal_line": 100, "track_width": 30}})
    E, S = len(seeds), n_steps
    actions = np.random.default_rng(action_seed).uniform(-1.0, 1.0, (E, S)).astype(np.float32)
    out = {k: [] for k in ("state", "new_state", "action", "reward", "terminal", "term", "done")}
    for e, seed in enumerate(seeds):
        np.random.seed(int(seed))
        env = be.BoatEnv(cfg, types.SimpleNamespace(experiment_dir=tempfile.mkdtemp()))
        rb = ReplayBuffer(S, (11,), 1)
        observation = env.reset()
        terms, dones = [], []
        for k in range(S):
            action = np.array([float(actions[e, k])], dtype=np.float64)
            observation_, reward, done, info = env.step(action)
            rb.store_transition(observation, action, reward, observation_,
                                info["termination"] == "reached_goal")     # main.py:83-88
            terms.append(TERM_CODES[info["termination"]] if done else 0)
            dones.append(bool(done))
            observation = env.reset() if done else observation_          # main.py:72
        out["state"].append(rb.state_memory)
        out["new_state"].append(rb.new_state_memory)
        out["action"].append(rb.action_memory)
        out["reward"].append(rb.reward_memory)
        out["terminal"].append(rb.terminal_memory)
        out["term"].append(terms)
        out["done"].append(dones)
    flat = {k: np.asarray(v) for k, v in out.items()}
    flat["term"] = flat["term"].astype(np.uint8)
    flat["done"] = flat["done"].astype(np.uint8)
    flat["seeds"], flat["actions"] = np.asarray(seeds, np.uint64), actions
    flat.update(_cfg_vector(cfg))
    path = os.path.join(HERE, "main_loop_goal.npz")
    np.savez_compressed(path, **flat)
    t = flat["term"]
    print(f"{path}: E={E} S={S} terms={np.bincount(t.ravel(), minlength=6).tolist()} "
          f"terminal={int(flat['terminal'].sum())} goal_steps={int((t == 1).sum())}")


def run_sac_learn(n_calls=2, batch=1024, seed=0):
    """ContinuousAgent.learn (continuous_agent.py:96-154) on fixed batches and noise."""
    import torch
    H.install_standins()
    import torch.nn.functional as F
    from agent.continuous_agent import ContinuousAgent  # reference module
    cfg = H.load_config()
    env = types.SimpleNamespace(action_space=sys_modules_box()(low=-1, high=1, dtype=np.float32))
    torch.manual_seed(seed)
    agent = ContinuousAgent(cfg, tempfile.mkdtemp(), (11,), env)
    rng = np.random.default_rng(seed + 17)
    batches = []
    for _ in range(n_calls):
        batches.append(dict(
            state=rng.uniform(0, 1, (batch, 11)),
            action=rng.uniform(-1, 1, (batch, 1)),
            reward=rng.standard_normal(batch) * 3,
            new_state=rng.uniform(0, 1, (batch, 11)),
            done=rng.random(batch) < 0.1))
    Normal = torch.distributions.Normal
    orig = (Normal.sample, Normal.rsample, F.mse_loss, torch.Tensor.backward)
    eps_log, mse_log, bwd_log = [], [], []
    gen = torch.Generator().manual_seed(seed + 99)

    def sample(self, sample_shape=torch.Size()):
        with torch.no_grad():
            eps = torch.randn(self._extended_shape(sample_shape), generator=gen)
            eps_log.append(eps.numpy().copy())
            return self.loc + eps * self.scale

    def rsample(self, sample_shape=torch.Size()):
        eps = torch.randn(self._extended_shape(sample_shape), generator=gen)
        eps_log.append(eps.numpy().copy())
        return self.loc + eps * self.scale

    def mse(a, b, *args, **kw):
        out = orig[2](a, b, *args, **kw)
        mse_log.append(float(out))
        return out

    def backward(self, *args, **kw):  # the loss each backward() starts from
        bwd_log.append(float(self.detach()))
        return orig[3](self, *args, **kw)

    Normal.sample, Normal.rsample, F.mse_loss = sample, rsample, mse
    torch.Tensor.backward = backward
    try:
        for b in batches:
            agent.memory.mem_cntr = agent.batch_size
            agent.memory.sample_buffer = (lambda bs, b=b: (b["state"], b["action"], b["reward"],
                                                           b["new_state"], b["done"]))
            agent.learn()
    finally:
        Normal.sample, Normal.rsample, F.mse_loss = orig[:3]
        torch.Tensor.backward = orig[3]
    # per call: value_loss, actor_loss, critic_loss (continuous_agent.py:123,138,150)
    out = {"n_calls": n_calls, "seed": seed, "eps": np.asarray(eps_log, np.float32),
           "mse": np.asarray(mse_log, np.float64), "backward_losses": np.asarray(bwd_log, np.float64)}
    for i, b in enumerate(batches):
        for k, v in b.items():
            out[f"b{i}_{k}"] = v
    for name in ("actor", "critic_1", "critic_2", "value", "target_value"):
        for k, v in getattr(agent, name).state_dict().items():
            out[f"w_{name}.{k}"] = v.numpy()
    out.update({f"cfg_{k}": np.asarray(v) for k, v in cfg["agent"].items()})
    path = os.path.join(HERE, "sac_learn.npz")
    np.savez_compressed(path, **out)
    print(f"{path}: calls={n_calls} eps={out['eps'].shape} mse={out['mse'].tolist()}")


# ---------------------------------------------------------------- long scripted runs
# Scripted rudder programs that reach the branches uniform / zero actions never reach
# (VERDICT r3 next 1): the heading past +-pi/2 (boat_env.py:110-111), the s_x < 0 half
# of out_of_bounds (:90), the default-t_max timeout after 10 000 steps (:98-101), and
# headings of hundreds of radians (the kernel's sincos argument reduction). Each program
# reads the reference boat's state and turns a wanted rudder angle into the action
# rudder += action / 10 needs (boat_env.py:72-73), clipped to the action space [-1, 1].
# The actions are recorded; the tests replay them open loop.

def _wrap(a):
    return (a + np.pi) % (2 * np.pi) - np.pi


def _heading_rudder(b, psi, kp=2.2, kd=450.0, lim=0.9):
    """PD on the heading s_r (yaw is a slow double integrator: I = 6e6, boat.yaml)."""
    return max(-lim, min(lim, kp * (psi - b.s_r) - kd * b.v_r))


def _action(b, rudder):
    return np.float32(max(-1.0, min(1.0, 10.0 * (rudder - b.rudder_angle))))


def prog_hold(rudder, n_hold):
    """Rudder to `rudder` (9 steps at |action| 1), held n_hold steps, then centred: the
    boat spins (|s_r| to ~240 rad), v_r grows to ~0.15 rad/s; still well conditioned.
    (Held for ~5 500 steps the reference's explicit Euler yaw runs away: 1-ulp changes
    in a transcendental grow past 1e-7 by step ~5 540 -- no implementation can match it
    there, so the hold ends at 4 500.)"""
    def pol(k, b):
        return _action(b, rudder if k < n_hold else 0.0)
    return pol


def prog_uturn(y0=-450.0):
    """Turn right to s_y < y0, then turn left to heading pi and hold it: the boat comes
    back across s_x = 0 inside the track (out_of_bounds by the s_x < 0 half of :90)."""
    st = {}

    def pol(k, b):
        if not st.get("turn"):
            if b.s_y < y0:
                st["turn"] = True
            else:
                return _action(b, _heading_rudder(b, -0.9))
        return _action(b, _heading_rudder(b, np.pi))
    return pol


def prog_orbit(ccw=True, r=250.0, box=(1000.0, 2000.0, 200.0)):
    """Steer around a rectangle of waypoints until the 10 000-step timeout; s_r winds
    up (ccw) or down (cw) by ~15 rad."""
    x0, x1, h = box
    pts = [(x0, -h), (x1, -h), (x1, h), (x0, h)] if ccw else [(x0, h), (x1, h), (x1, -h), (x0, -h)]
    st = {"i": 0}

    def pol(k, b):
        tx, ty = pts[st["i"] % 4]
        if np.hypot(tx - b.s_x, ty - b.s_y) < r:
            st["i"] += 1
            tx, ty = pts[st["i"] % 4]
        psi = b.s_r + _wrap(np.arctan2(ty - b.s_y, tx - b.s_x) - b.s_r)
        return _action(b, _heading_rudder(b, psi))
    return pol


def prog_slalom(amp=1.8):
    """Heading oscillating between -amp and +amp (past -pi/2 and +pi/2 in one episode);
    needs a wide track (the swings drift ~2 400 m sideways)."""
    st = {"sg": -1}

    def pol(k, b):
        if st["sg"] * b.s_r > amp - 0.05:
            st["sg"] = -st["sg"]
        return _action(b, _heading_rudder(b, st["sg"] * amp))
    return pol


LONG_STEPS = 10000


def run_long(name, overrides, programs, seeds, n_steps=LONG_STEPS, every=10):
    """Like run_seeded, with one scripted program per env (restarted after every reset).
    Every step keeps term, done and the f64 reward; the full state, obs, wind and
    episode reward are kept at a subset of steps (every `every`-th, every 128th, and the
    steps around each episode end) to hold the file near 1 MB."""
    be = H.boat_env_module()
    cfg = H.load_config(overrides)
    E, S = len(seeds), n_steps
    oob = float(cfg.boat_env.track_width) + float(cfg.boat_env.boat_out_of_bounds_offset)
    actions = np.zeros((E, S), np.float32)
    full = {k: np.zeros((E, S) + sh, dt) for k, sh, dt in (
        ("reward", (), np.float64), ("done", (), np.uint8), ("term", (), np.uint8),
        ("state", (len(STATE_FIELDS),), np.float64), ("obs", (11,), np.float64),
        ("wind", (2,), np.float64), ("ep_reward", (), np.float64),
        ("reset_obs", (11,), np.float64), ("reset_state", (len(STATE_FIELDS),), np.float64),
        ("start_y", (), np.int32))}
    full["reset_obs"][:] = np.nan
    full["reset_state"][:] = np.nan
    init = {"init_obs": [], "init_state": [], "init_start_y": []}
    counters = []
    hits = {"heading_pos": 0, "heading_neg": 0, "rudder_penalty": 0, "oob_sx_neg": 0,
            "timeout_default": 0, "max_abs_s_r": 0.0}
    for e, seed in enumerate(seeds):
        np.random.seed(int(seed))
        env = be.BoatEnv(cfg, types.SimpleNamespace(experiment_dir=tempfile.mkdtemp()))
        obs0 = env.reset()
        init["init_obs"].append(np.asarray(obs0, np.float64))
        init["init_state"].append(_state(env.boat))
        init["init_start_y"].append(int(env.boat.s_y_start))
        pol = programs[e]()
        for k in range(S):
            b = env.boat
            wv, wa = b.wind.get_wind(b.index)
            a = pol(k, b)
            actions[e, k] = a
            o, r, d, info = env.step(np.array([float(a)], dtype=np.float64))
            b = env.boat
            full["wind"][e, k] = (float(wv), float(wa))
            full["obs"][e, k] = np.asarray(o, np.float64)
            full["reward"][e, k] = float(r)
            full["done"][e, k] = bool(d)
            full["term"][e, k] = TERM_CODES[info["termination"]] if d else 0
            full["state"][e, k] = _state(b)
            full["ep_reward"][e, k] = float(info["episode_reward"])
            hits["heading_pos"] += int(b.s_r > np.pi / 2)
            hits["heading_neg"] += int(b.s_r < -np.pi / 2)
            hits["rudder_penalty"] += int(abs(b.rudder_angle) > np.pi / 4)
            hits["max_abs_s_r"] = max(hits["max_abs_s_r"], abs(float(b.s_r)))
            if d and info["termination"] == "out_of_bounds" and b.s_x < 0 and abs(b.s_y) <= oob:
                hits["oob_sx_neg"] += 1
            if d and info["termination"] == "timeout" and b.index == int(cfg.base_settings.t_max
                                                                      / cfg.base_settings.dt):
                hits["timeout_default"] += 1
            if d:
                ro = env.reset()
                full["reset_obs"][e, k] = np.asarray(ro, np.float64)
                full["reset_state"][e, k] = _state(env.boat)
                full["start_y"][e, k] = int(env.boat.s_y_start)
                pol = programs[e]()
        counters.append([env.info[k] for k in ("reached_goal", "out_of_bounds", "out_of_fuel",
                                                "rudder_broken", "timeout")])
    ks = np.arange(S)
    near = np.zeros(S, bool)
    for dk in (-1, 0, 1):
        near |= np.roll(full["done"].any(0), dk)
    keep = np.flatnonzero((ks % every == every - 1) | (ks % 128 == 127) | near | (ks < 8))
    out = {"keep": keep.astype(np.int32), "reward": full["reward"], "done": full["done"],
           "term": full["term"], "actions": actions, "seeds": np.asarray(seeds, np.uint64),
           "state_fields": np.array(STATE_FIELDS), "counters": np.asarray(counters),
           "n_steps": np.int32(S)}
    for k in ("state", "obs", "wind", "ep_reward", "reset_obs", "reset_state", "start_y"):
        out[k] = full[k][:, keep]
    for k, v in init.items():
        out[k] = np.asarray(v)
    out.update({f"hits_{k}": np.asarray(v) for k, v in hits.items()})
    out.update(_cfg_vector(cfg))
    path = os.path.join(HERE, f"long_{name}.npz")
    np.savez_compressed(path, **out)
    print(f"{path}: E={E} S={S} kept={len(keep)} "
          f"terms={np.bincount(full['term'].ravel(), minlength=6).tolist()} hits={hits}")


def make_long():
    base = {"experiment": 1, "test_mode": 0}
    progs = [lambda: prog_hold(0.9, 4500), prog_uturn, lambda: prog_orbit(True),
             lambda: prog_orbit(False)]
    run_long("exp1", {"base_settings": dict(base)}, progs, SEEDS[:4])
    progs6 = [lambda: prog_hold(-0.9, 4500), prog_uturn, lambda: prog_orbit(True),
              lambda: prog_orbit(False)]
    run_long("exp6", {"base_settings": dict(base, experiment=6)}, progs6,
             np.array([3, 0, 1, 2**32 - 1], np.uint64))
    run_long("exp6_slalom", {"base_settings": dict(base, experiment=6),
                             "boat_env": {"track_width": 3000}},
             [prog_slalom, prog_slalom], np.array([5, 12345], np.uint64))


def make_long_wind1():
    """Round 4: the one-curve wind experiments on the same programs (exp 4: the
    speed curve; exp 5: the rectified angle), default configs."""
    base = {"experiment": 4, "test_mode": 0}
    run_long("exp4", {"base_settings": dict(base)}, [lambda: prog_hold(0.9, 4500), prog_uturn],
             np.array([7, 2**31 + 5], np.uint64))
    run_long("exp5", {"base_settings": dict(base, experiment=5)},
             [lambda: prog_hold(-0.9, 4500), lambda: prog_orbit(True)], np.array([9, 123456789], np.uint64))


def sys_modules_box():
    import sys
    return sys.modules["gym.spaces"].Box


def main():
    import sys
    if sys.argv[1:] == ["sac"]:
        run_sac_learn()
        return
    if sys.argv[1:] == ["main_loop"]:
        run_main_loop()
        return
    if sys.argv[1:] == ["toys"]:
        run_toys()
        return
    if sys.argv[1:] == ["replay"]:
        run_replay()
        return
    if sys.argv[1:] == ["long"]:
        make_long()
        make_long_wind1()
        return
    if sys.argv[1:] == ["long_wind1"]:
        make_long_wind1()
        return
    run_toys()
    run_replay()
    run_main_loop()
    run_sac_learn()
    make_long()
    make_long_wind1()
    for exp in range(1, 7):
        run_seeded(f"exp{exp}_uniform", {"base_settings": {"experiment": exp, "test_mode": 0}},
                   400, "uniform", action_seed=100 + exp)
    run_seeded("exp6_narrow", {"base_settings": {"experiment": 6, "test_mode": 0},
                               "boat_env": {"track_width": 20}}, 700, "uniform", action_seed=7)
    run_seeded("exp2_narrow", {"base_settings": {"experiment": 2, "test_mode": 0},
                               "boat_env": {"track_width": 20}}, 500, "uniform", action_seed=8)
    run_seeded("exp6_fuel", {"base_settings": {"experiment": 6, "test_mode": 1},
                             "boat": {"fuel": 30}}, 100, "zero")
    run_seeded("exp6_timeout", {"base_settings": {"experiment": 6, "test_mode": 1, "t_max": 5}},
               60, "zero")
    run_seeded("exp5_timeout", {"base_settings": {"experiment": 5, "test_mode": 0, "t_max": 5}},
               60, "uniform", action_seed=9)
    run_seeded("exp6_goal", {"base_settings": {"experiment": 6, "test_mode": 1},
                             "boat_env": {"goal_line": 100}}, 400, "zero")
    run_seeded("exp3_big", {"base_settings": {"experiment": 3, "test_mode": 0}},
               60, "big", action_seed=10)
    for exp in (4, 5, 6):
        run_wind(exp)
    run_wind(6, n_seeds=32, t_max=5)
    for exp in range(1, 7):
        convert_recorded(exp)


if __name__ == "__main__":
    main()
