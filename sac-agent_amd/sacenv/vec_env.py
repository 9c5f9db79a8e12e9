"""VecBoatEnv: N boat envs per GPU behind the reference's Gym surface.

Batched counterpart of ``BoatEnv`` (environment/boat_env.py:9-140). Every
env is an independent reference ``BoatEnv`` with its own numpy-legacy RNG
stream: env ``e`` seeded with ``s`` behaves exactly like
``np.random.seed(s); env = BoatEnv(cfg)`` in the reference — the constructor
builds one Boat (boat_env.py:15) and every ``reset`` another (:121).

All compute runs in libsacenv.so (gfx950 HIP). The env's whole state lives in
one device arena (a uint8 tensor) whose fields are exposed here as tensor
views; ``step`` enqueues one kernel on the current torch stream and never
synchronises.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _lib
from .config import BoatConfig, make_params, observation_bounds, t_from_index
from .spaces import Box

RECORD_BYTES = _lib.RECORD_BYTES  # packed per-env record: obs f32x11 | reward f32 | done u8 | term u8


class VecBoatEnv:
    """``num_envs`` boat envs resident on one GPU.

    Parameters
    ----------
    config : reference-style config (YAML path, dict, DotMap) or BoatConfig.
    num_envs : envs on this device.
    seed : base seed; env ``e`` gets ``seeds[e] = (seed + env_id_offset + e) mod 2**32``
        unless ``seeds`` is given explicitly.
    max_episode_steps : >0 truncates episodes (term code 6) after that many steps.
    autoreset : start the next episode inside ``step`` for envs that end
        (gym vector-env semantics: the returned obs row is the new episode's
        first obs, the terminal obs is ``info['final_obs']``). Episodes are
        pre-drawn up to 256 ahead per env (``_lib.SLOTS``), from the env's own
        RNG stream in the reference's order, so draws match the reference
        exactly; a refill launch tops the slots up (see ``refill``).
    env_id_offset : global id of this rank's first env (multi-GPU sharding).
    record_knots / record_accel / record_reward64 : extra outputs (tests, shim).
    wind_table : [2, int(t_max/dt)] recorded wind (velocity, angle) for all envs.
    n_helpers : autoreset: workgroups of a refill's draw launch (four envs' draws each at a
        time); default: 3/16 of the padded env count (at least 1 024).
    auto_refill : autoreset: launch ``refill()`` after every ``_lib.REFILL_PERIOD``-th
        step issued through this object. Pass False when capturing steps into a
        graph and place ``refill()`` yourself (at most REFILL_PERIOD steps apart).
    """

    def __init__(self, config=None, num_envs: int = 1, *, seed: int = 0, seeds=None,
                 device=None, max_episode_steps: int = 0, autoreset: bool = True,
                 env_id_offset: int = 0, record_knots: bool = False, record_accel: bool = False,
                 record_reward64: bool = False, wind_table=None, n_helpers: int | None = None,
                 auto_refill: bool = True):
        self.lib = _lib.load()
        self.cfg = BoatConfig.from_any(config)
        self.num_envs = N = int(num_envs)
        if N <= 0:
            raise ValueError("num_envs must be positive")
        self.device = torch.device(device if device is not None else "cuda")
        if self.device.type != "cuda":
            raise RuntimeError("VecBoatEnv runs on a GPU (HIP); no CPU path")
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.env_id_offset = int(env_id_offset)
        self.autoreset = bool(autoreset)
        self.auto_refill = bool(auto_refill)
        self._since_refill = 0
        if n_helpers is None:
            # one 16-lane draw group (4 per helper wave) per env a refill typically lists (~3 of
            # 4 after a 256-step segment): 12 288 at 65 536 envs; measured 45.6-45.7 G
            # env-steps/s against 45.1-45.2 with 8 192 and 44.1 with 4 096 (more: the same)
            n_helpers = max(1024, ((N + 63) // 64 * 64) * 3 // 16)
        flags = ((_lib.OUT_KNOTS if record_knots else 0) | (_lib.OUT_ACCEL if record_accel else 0)
                 | (_lib.OUT_REWARD64 if record_reward64 else 0))
        self.params = make_params(self.cfg, N, max_episode_steps=max_episode_steps,
                                  autoreset=autoreset, n_helpers=n_helpers, out_flags=flags,
                                  use_wind_table=wind_table is not None)
        self._pp = C.byref(self.params)
        self.layout = L = _lib.layout(self.params)
        self.n_pad = NP = int(L.n_pad)
        self.arena = torch.zeros(int(L.total_bytes), dtype=torch.uint8, device=self.device)
        nk = int(self.cfg.fixed_points)

        def view(off, dtype, *shape):
            esz = torch.empty((), dtype=dtype).element_size()
            cnt = int(np.prod(shape))
            return self.arena[off: off + cnt * esz].view(dtype).view(*shape)

        f64, i32 = torch.float64, torch.int32

        def pair_view(off):  # paired f64 fields: [n_pad][2] blocks, env stride 16 B
            k = (off % 16) // 8
            return view(off - 8 * k, f64, NP, 2)[:N, k]

        # carried state (strided views of the paired fields, first N envs)
        for name in ("s_x", "s_y", "s_r", "v_x", "v_y", "v_r", "rudder", "ep_reward"):
            setattr(self, name, pair_view(getattr(L, name)))
        self._t_view = view(L.t, f64, NP)[:N]
        self._t_from_index = t_from_index(float(self.cfg.dt))
        self.index = view(L.index, i32, NP)[:N]
        self.cons = view(L.cons, i32, NP)[:N]
        # RAW arena words (ABI 18+): bits 0..15 the MT word index, bit 16 the refill's
        # pre-twisted mt_next flag; between a refill's draw and fit launches the index can
        # point past 623 into mt_next. `mt_index` is the stream position a host should read.
        self.mt_pos = view(L.mt_pos, i32, NP)[:N]
        self.start_y_slots = view(L.start_y, i32, _lib.SLOTS, NP)[:, :N]
        self.counters = view(L.counters, i32, _lib.N_COUNTERS, NP)[:, :N]
        # info['termination'] as the reference keeps it: the last code 1..5 (0: none yet)
        self.last_term = view(L.last_term, i32, NP)[:N]
        self.wind_knots = view(L.wind_knots, f64, NP, _lib.SLOTS, 2, nk, 2)
        # the drawn knots per slot exist only with record_knots (SACENV_OUT_KNOTS)
        self.knots_raw_slots = view(L.knots_raw, f64, NP, _lib.SLOTS, 2, nk) if record_knots else None
        self.mt_key = view(L.mt_key, i32, NP, _lib.MT_N)[:N]
        # the block after mt_key, twisted ahead by each refill (valid while mt_pos bit 16 is set)
        self.mt_next = view(L.mt_next, i32, NP, _lib.MT_N)[:N]
        self.spline_g = view(L.spline_g, f64, nk, nk)
        # outputs: the packed record (the all-gather payload) and extras
        self.record = self.arena[L.record: L.record + RECORD_BYTES * NP]
        self.obs = view(L.obs, torch.float32, NP, _lib.OBS_DIM)[:N]
        self.reward = view(L.reward, torch.float32, NP)[:N]
        self.done = view(L.done, torch.uint8, NP)[:N]
        self.term = view(L.term, torch.uint8, NP)[:N]
        self.final_obs = view(L.final_obs, torch.float32, NP, _lib.OBS_DIM)[:N]
        # the terminal-obs region as raw bytes (n_pad rows): a pooled transition's s'
        self.final_obs_bytes = self.arena[L.final_obs: L.final_obs + 4 * _lib.OBS_DIM * NP]
        self.final_ep_reward = view(L.final_ep_reward, f64, NP)[:N]
        self.accel = view(L.accel, f64, 3, NP)[:, :N]
        self.reward64 = view(L.reward64, f64, NP)[:N]
        self.status = view(L.status, i32, 64)        # [0] refills done, [1] status bits
        if wind_table is not None:
            wt = torch.as_tensor(np.asarray(wind_table, np.float64).reshape(2, -1))
            if wt.shape[1] != self.cfg.wind_len:
                raise ValueError("wind_table must be [2, int(t_max/dt)]")
            view(L.wind_table, f64, 2, self.cfg.wind_len).copy_(wt)

        # Gym surface (boat_env.py:37-65)
        self.action_space = Box(low=-1, high=1, dtype=np.float32)
        low, high = observation_bounds()
        self.observation_space = Box(low=low, high=high, dtype=np.float32)

        if seeds is None:
            gid = np.arange(N, dtype=np.uint64) + np.uint64(self.env_id_offset)
            seeds = (np.uint64(seed) + gid) & np.uint64(0xFFFFFFFF)
        seeds = np.asarray(seeds, dtype=np.uint64)
        if seeds.shape != (N,):
            raise ValueError("seeds must have one entry per env")
        if np.any(seeds > 0xFFFFFFFF):
            raise ValueError("Seed must be between 0 and 2**32 - 1")
        self.seeds = seeds
        self._seeds_dev = torch.from_numpy(seeds.astype(np.uint32).view(np.int32)).to(self.device)
        # np.random.seed + BoatEnv.__init__'s Boat (boat_env.py:15)
        _lib.check(self.lib.sacenv_boat_init(self._pp, self._ptr, self._seeds_dev.data_ptr(),
                                             self.stream))

    # ------------------------------------------------------------------ plumbing
    @property
    def mt_index(self) -> torch.Tensor:
        """Each env's MT19937 stream position: the raw ``mt_pos`` word without its flag bit
        -- the next word's index in ``mt_key``, 0..624 as numpy's ``get_state()[2]`` (624:
        twist first). Only between a refill's draw and fit launches can it exceed 624 (the
        draws went on into the pre-twisted ``mt_next``; the fit makes that block current).
        Synchronise before reading it on the host."""
        return self.mt_pos & 0xFFFF

    @property
    def _ptr(self) -> int:
        return self.arena.data_ptr()

    @property
    def stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    @property
    def t(self) -> torch.Tensor:
        """Boat.t of each env: index * dt when dt makes ``t += dt`` exact (the kernel
        then carries no t), else the carried f64 field."""
        if self._t_from_index:
            return self.index.to(torch.float64) * float(self.cfg.dt)
        return self._t_view

    @property
    def start_y(self) -> torch.Tensor:
        """Boat.s_y_start of each env's current episode."""
        slot = (self.cons % _lib.SLOTS).long() if self.autoreset else torch.zeros_like(self.cons).long()
        return self.start_y_slots.gather(0, slot[None, :])[0]

    @property
    def knots_raw(self) -> torch.Tensor:
        """Knot values [2, n_knots, N] of each env's current episode (record_knots)."""
        if self.knots_raw_slots is None:
            raise RuntimeError("construct the env with record_knots=True to keep the drawn knots")
        slot = (self.cons % _lib.SLOTS).long() if self.autoreset else torch.zeros_like(self.cons).long()
        k = self.knots_raw_slots[: self.num_envs]                     # [N, SLOTS, 2, nk]
        return k[torch.arange(self.num_envs, device=k.device), slot].permute(1, 2, 0)

    # ------------------------------------------------------------------ gym API
    def reset(self, env_ids=None) -> torch.Tensor:
        """BoatEnv.reset for all envs, or for ``env_ids`` (boat_env.py:120-126)."""
        if env_ids is None:
            _lib.check(self.lib.sacenv_boat_reset(self._pp, self._ptr, None, 0, self.stream))
        else:
            ids = torch.as_tensor(env_ids, dtype=torch.int32, device=self.device).contiguous()
            if ids.numel():
                _lib.check(self.lib.sacenv_boat_reset(self._pp, self._ptr, ids.data_ptr(),
                                                      ids.numel(), self.stream))
                self._keep = ids
        return self.obs

    def compact_done(self, done=None):
        """(ids, count) device tensors: the envs whose ``done`` byte is set, ascending
        (done-mask compaction on the GPU; no host round trip)."""
        d = self.done if done is None else torch.as_tensor(done, dtype=torch.uint8, device=self.device)
        d = d.contiguous()
        ids = torch.empty(d.numel(), dtype=torch.int32, device=self.device)
        count = torch.empty(1, dtype=torch.int32, device=self.device)
        _lib.check(self.lib.sacenv_compact_done(d.data_ptr(), d.numel(), ids.data_ptr(),
                                                count.data_ptr(), self.stream))
        self._keep_c = d
        return ids, count

    def reset_done(self, done=None) -> torch.Tensor:
        """BoatEnv.reset for every env whose ``done`` byte is set (default: the last
        step's done mask), entirely on the device: compaction + reset of the list."""
        ids, count = self.compact_done(done)
        _lib.check(self.lib.sacenv_boat_reset_list(self._pp, self._ptr, ids.data_ptr(),
                                                   count.data_ptr(), self.stream))
        self._keep = (ids, count)
        return self.obs

    def reset_explicit(self, env_ids, start_y, knots=None) -> torch.Tensor:
        """Reset with caller-supplied draws (replaying recorded episodes; autoreset=False)."""
        ids = torch.as_tensor(env_ids, dtype=torch.int32, device=self.device).contiguous()
        sy = torch.as_tensor(start_y, dtype=torch.int32, device=self.device).contiguous()
        kn = None
        if knots is not None:
            kn = torch.as_tensor(knots, dtype=torch.float64, device=self.device).contiguous()
        _lib.check(self.lib.sacenv_boat_reset_explicit(
            self._pp, self._ptr, ids.data_ptr(), ids.numel(), sy.data_ptr(),
            None if kn is None else kn.data_ptr(), self.stream))
        self._keep = (ids, sy, kn)  # alive until the stream has consumed them
        return self.obs

    def check_actions(self, actions: torch.Tensor) -> None:
        """The kernel reads num_envs f32 values from the pointer: refuse anything else
        (a wrong tensor would otherwise be an out-of-bounds device read)."""
        if not isinstance(actions, torch.Tensor):
            raise TypeError("actions must be a torch tensor on the env's device")
        if actions.dtype != torch.float32 or not actions.is_contiguous():
            raise ValueError("actions must be a contiguous float32 tensor")
        if actions.numel() != self.num_envs:
            raise ValueError(f"actions must hold num_envs={self.num_envs} values, got {actions.numel()}")
        if actions.device != self.device:
            raise ValueError(f"actions are on {actions.device}, the env on {self.device}")

    def step_async(self, actions: torch.Tensor) -> None:
        """Enqueue one step; ``actions`` is a contiguous f32 device tensor of N values."""
        self.check_actions(actions)
        _lib.check(self.lib.sacenv_boat_step(self._pp, self._ptr, actions.data_ptr(), self.stream))
        self._after_step()

    def step_pooled_async(self, actions: torch.Tensor, trans_row: torch.Tensor) -> None:
        """``step_async`` that also writes the step's transition row (s', reward,
        action, term, and obs3_next in experiment 2; ``sacenv_boat_step_pooled``,
        ``sacenv.dist.TransitionLayout``) into ``trans_row``, a 16-B aligned uint8
        device tensor of ``_lib.trans_bytes(experiment) * n_pad`` bytes (e.g. a row
        of a pooling buffer: no copy launches)."""
        self.check_actions(actions)
        nb = _lib.trans_bytes(self.params.experiment) * self.n_pad
        if (trans_row.dtype != torch.uint8 or trans_row.device != self.device
                or trans_row.numel() != nb or not trans_row.is_contiguous()):
            raise ValueError(f"trans_row must be a contiguous uint8 device tensor of {nb} bytes")
        _lib.check(self.lib.sacenv_boat_step_pooled(self._pp, self._ptr, actions.data_ptr(),
                                                    trans_row.data_ptr(), self.stream))
        self._after_step()

    def first_obs_template(self) -> torch.Tensor:
        """The first obs of a fresh Boat (boat_env.py:152-198 -> return_state) as the
        kernel writes it, f32 [11]; entry 3 (normalised s_y) depends on the start y in
        experiment 2 (the transition row's obs3_next carries it)."""
        from .config import first_obs_template
        return torch.from_numpy(first_obs_template(self.cfg))

    def rollout(self, actions, records=None, final_obs=None):
        """``K`` steps in one launch for an open-loop action sequence ``actions``
        [K, N] (f32, device): the same results as K ``step`` calls, bit for bit.
        Returns ``records`` (u8 [K, 50 n_pad], step k's packed record; views via
        ``record_views``) and ``final_obs`` (f32 [K, n_pad, 11] or None: terminal
        obs where step k's done is set). The env's own record is not written."""
        a = torch.as_tensor(actions, device=self.device)
        if a.dtype != torch.float32:
            a = a.to(torch.float32)
        K = int(a.shape[0])
        a = a.reshape(K, self.num_envs).contiguous()
        if self.autoreset and K > _lib.REFILL_PERIOD:
            raise ValueError(f"rollout of more than {_lib.REFILL_PERIOD} steps in autoreset mode")
        if self.autoreset and self.auto_refill and self._since_refill + K > _lib.REFILL_PERIOD:
            self.refill()
        if records is None:
            records = torch.empty((K, RECORD_BYTES * self.n_pad), dtype=torch.uint8, device=self.device)
        _lib.check(self.lib.sacenv_boat_rollout(
            self._pp, self._ptr, a.data_ptr(), K, records.data_ptr(),
            None if final_obs is None else final_obs.data_ptr(), self.stream))
        self._keep_roll = a
        if self.autoreset:
            self._since_refill += K
        return records, final_obs

    def segment_async(self, actions: torch.Tensor, n_steps: int | None = None, *, act_ready=None,
                      step_done=None, seq0: int = 0, trans=None, trans_stride: int = 0, stage=None,
                      stage_marks=None) -> None:
        """``n_steps`` BoatEnv.step calls in ONE persistent launch (``sacenv_boat_segment``):
        the same results as ``n_steps`` ``step_async`` calls, bit for bit, with the
        carried state in registers between the steps and each step's outputs in the
        env's record / final_obs (as ``step``). ``actions`` is a [K >= n_steps, N] f32
        device tensor whose rows may be strided (e.g. rows of a larger table).

        Closed-loop hand-off per owner wave (64 envs): with ``act_ready`` (u32 device
        [n_pad/64]) the wave steps ks only once ``act_ready[w] >= seq0 + ks + 1``;
        with ``step_done`` it publishes ``seq0 + ks + 1`` there once step ks's outputs
        are visible. ``trans`` (u8 device, 16-B aligned): step ks's pooled transition
        row at ``trans[ks * trans_stride:]``. ``stage`` / ``stage_marks``: the staged
        replay rows (env-major: env e's 64-B row of step ks at ``(e * K + ks) * 64``),
        written where bit ks % 64 of ``stage_marks[e * ceil(K / 64) + ks // 64]`` is set
        (int64 [n_pad, ceil(K / 64)]; consumed: the launch clears them; K <= 256);
        ``sacenv.replay.StagedReplay``."""
        K = int(actions.shape[0]) if n_steps is None else int(n_steps)
        if (not isinstance(actions, torch.Tensor) or actions.dtype != torch.float32
                or actions.device != self.device or actions.dim() != 2
                or actions.shape[1] != self.num_envs or actions.stride(1) != 1 or actions.shape[0] < K):
            raise ValueError(f"actions must be a float32 [>= {K}, {self.num_envs}] device tensor with "
                             "contiguous rows")
        if self.autoreset and K > _lib.REFILL_PERIOD:
            raise ValueError(f"a segment of more than {_lib.REFILL_PERIOD} steps in autoreset mode")
        if self.autoreset and self.auto_refill and self._since_refill + K > _lib.REFILL_PERIOD:
            self.refill()
        nw = self.n_pad // 64
        for name, f in (("act_ready", act_ready), ("step_done", step_done)):
            if f is not None and (f.dtype not in (torch.int32, torch.uint32) or f.numel() < nw
                                  or f.device != self.device or not f.is_contiguous()):
                raise ValueError(f"{name} must be a contiguous 32-bit device tensor of n_pad/64 = {nw}")
        if trans is not None:
            nb = _lib.trans_bytes(self.params.experiment) * self.n_pad
            if (trans.dtype != torch.uint8 or trans.device != self.device or not trans.is_contiguous()
                    or trans.numel() < (K - 1) * int(trans_stride) + nb):
                raise ValueError("trans must be a contiguous uint8 device tensor holding K rows")
        if stage is not None:
            if (stage.dtype != torch.uint8 or stage.device != self.device or not stage.is_contiguous()
                    or stage.numel() < K * 64 * self.n_pad):
                raise ValueError("stage must be a contiguous uint8 device tensor of n_steps x 64 x n_pad bytes")
            if stage_marks is not None and (stage_marks.dtype != torch.int64 or stage_marks.device != self.device
                                            or not stage_marks.is_contiguous()
                                            or stage_marks.numel() < self.n_pad * -(-K // 64)):
                raise ValueError("stage_marks must be a contiguous int64 device tensor of n_pad x ceil(n_steps/64)")
        _lib.check(self.lib.sacenv_boat_segment(
            self._pp, self._ptr, actions.data_ptr(), int(actions.stride(0)), K,
            None if act_ready is None else act_ready.data_ptr(),
            None if step_done is None else step_done.data_ptr(), int(seq0) & 0xFFFFFFFF,
            None if trans is None else trans.data_ptr(), int(trans_stride),
            None if stage is None else stage.data_ptr(), None if stage_marks is None else stage_marks.data_ptr(),
            self.stream))
        self._keep_seg = (actions, act_ready, step_done, trans, stage, stage_marks)
        if self.autoreset:
            self._since_refill += K

    def record_views(self, rec: torch.Tensor):
        """(obs [N, 11], reward [N], done [N], term [N]) views of one packed record."""
        NP, N = self.n_pad, self.num_envs
        obs = rec[: 44 * NP].view(torch.float32).view(NP, _lib.OBS_DIM)[:N]
        return (obs, rec[44 * NP: 48 * NP].view(torch.float32)[:N], rec[48 * NP: 49 * NP][:N],
                rec[49 * NP: 50 * NP][:N])

    def _after_step(self) -> None:
        if self.autoreset:
            self._since_refill += 1
            if self.auto_refill and self._since_refill >= _lib.REFILL_PERIOD:
                self.refill()

    def refill(self) -> None:
        """Enqueue the slot refill (autoreset): draw and fit the replacement episodes of
        every env that ended since the last refill. Needed at least every
        ``_lib.REFILL_PERIOD`` steps; ``auto_refill`` does it for eager stepping."""
        _lib.check(self.lib.sacenv_boat_refill(self._pp, self._ptr, self.stream))
        self._since_refill = 0

    def check_status(self) -> None:
        """Raise if the device flagged an error (synchronises): an env that restarted
        past its pre-drawn episodes (refills further apart than REFILL_PERIOD steps)."""
        bits = int(self.status[1].item())
        if bits & _lib.STATUS_SLOT_UNDERFLOW:
            raise _lib.SacenvError("slot underflow: more than REFILL_PERIOD steps without refill()")
        if bits & _lib.STATUS_LIST_TIMEOUT:
            raise _lib.SacenvError("refill listing timed out: a listing workgroup never published")
        if bits & _lib.STATUS_HANDOFF_TIMEOUT:
            raise _lib.SacenvError("segment hand-off timed out: an action row's flag never came; "
                                   "hand-off launches on this arena now step nothing")

    def step(self, actions):
        """BoatEnv.step for all envs (boat_env.py:67-115).

        Returns ``(obs, reward, done, info)`` as device tensors that alias the
        env's output buffers (overwritten by the next step; clone to keep).
        ``info`` holds ``term`` (SACENV_TERM_* codes; 1..5 in the order of the
        reference info-dict keys), ``final_obs`` and ``final_ep_reward``
        (valid where done) and the cumulative ``counters`` [5, N].
        """
        a = torch.as_tensor(actions, device=self.device)
        if a.dtype != torch.float32:
            a = a.to(torch.float32)
        a = a.reshape(self.num_envs).contiguous()
        self._last_action = a
        self.step_async(a)
        info = {"term": self.term, "final_obs": self.final_obs,
                "final_ep_reward": self.final_ep_reward, "counters": self.counters}
        return self.obs, self.reward, self.done, info

    def wind_eval(self, env_ids, idx):
        """Wind.get_wind(index) of each env's current episode -> (velocity, angle) f64."""
        ids = torch.as_tensor(env_ids, dtype=torch.int32, device=self.device).contiguous()
        ix = torch.as_tensor(idx, dtype=torch.int32, device=self.device).contiguous()
        if ids.shape != ix.shape:
            raise ValueError("env_ids and idx must have the same shape")
        v = torch.empty(ids.shape, dtype=torch.float64, device=self.device)
        a = torch.empty_like(v)
        _lib.check(self.lib.sacenv_boat_wind_eval(self._pp, self._ptr, ids.data_ptr(),
                                                  ix.data_ptr(), ids.numel(), v.data_ptr(),
                                                  a.data_ptr(), self.stream))
        self._keep = (ids, ix)
        return v, a

    def state_dict(self) -> dict:
        """Host copy of the carried state (parity tests / checkpoints)."""
        torch.cuda.synchronize(self.device)
        d = {k: getattr(self, k).cpu().numpy() for k in
             ("s_x", "s_y", "s_r", "v_x", "v_y", "v_r", "rudder", "t", "ep_reward", "index")}
        d["start_y"] = self.start_y.cpu().numpy()
        d["fuel"] = int(self.cfg.fuel) - d["index"].astype(np.int64)
        d["a_x"], d["a_y"], d["a_r"] = self.accel.cpu().numpy()
        return d

    @property
    def counters_dict(self) -> dict:
        c = self.counters.cpu().numpy().astype(np.int64)
        return {name: c[k] for k, name in enumerate(_lib.TERM_NAMES[1:6])}
