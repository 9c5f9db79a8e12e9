"""The acting loop of main.py:70-91 -- ``choose_action`` then ``env.step`` -- as two
device-side pipelines handing off through per-owner-wave flags.

The env runs as persistent segment launches (``VecBoatEnv.segment_async``,
``sacenv_boat_segment``: up to 256 steps per launch, the carried state in
registers), the policy as ``NativeSAC.choose_action_handoff`` launches on a second
stream. For owner wave w (64 envs) and sequence number q:

    policy row q  waits  step_done[w] >= q      (the obs of step q-1, or the reset obs)
                  writes actions[q % K][64w .. 64w+63]
                  then   act_ready[w] = q + 1
    env step q    waits  act_ready[w] >= q + 1
                  writes the record (obs, reward, done, term) and final_obs
                  then   step_done[w] = q + 1

so no host synchronisation and no launch boundary sits between two env steps,
and each wave proceeds as soon as ITS policy rows are ready. The env's single
record is safe: step q+1 cannot overwrite step q's obs before the policy read
them (it waits for the row the policy writes after reading). Results equal the
eager loop ``a = agent.choose_action(env.obs, eps); env.step_async(a)`` bit for
bit (``test_closed_loop_equals_eager_loop`` in tests/test_segment_gpu.py).

Co-residency. The hand-off makes progress only if every owner wave of the
segment launch is resident while policy workgroups spin beside it: a policy
workgroup waits for its own owner wave, owner waves never leave before the
segment ends, and the policy's next launch starts only when the whole previous
one is done. So the plan (``make_plan``, from both kernels' VGPRs and LDS as the
library reports them through the C ABI) requires
  * every owner wave to fit on the device at once with room left, on every
    SIMD, for one policy wave (VGPRs: a SIMD holds 512 per lane, allocated in
    granules of 8; wave slots: 8 per SIMD), and the CU's LDS to hold its owner
    waves plus one policy workgroup;
  * at most ONE policy workgroup per CU: the hand-off act kernel is launched with
    its LDS padded past half a CU's 160 KB, so no arrangement of dispatched
    policy workgroups can keep an owner wave out.
Then all owner waves are resident, each policy workgroup's wait ends, and the
policy launches drain. A configuration that fails is refused (65 536 envs fit:
one owner wave of ~320 VGPRs per SIMD beside one ~152-VGPR policy wave).

Which form runs. ``ClosedLoop(env, agent)`` runs the EAGER form
by default (``run_eager``: one ``choose_action`` launch at full occupancy, then one
step launch, on one stream -- main.py:78-81's order, bit-identical to the hand-off):
with the reference's 256-256 actor on 65 536 envs the policy (~75 us) dwarfs the env
step (~1.3 us), the launch boundary the hand-off removes costs nothing by comparison,
and the hand-off's policy -- one workgroup per CU beside the resident owner waves --
runs at 0.43x its full-occupancy rate (measured 0.38 G vs 0.80 G env-steps/s). The
hand-off form (``handoff=True``) pays where the policy is cheaper than the env step
(a small actor, or far more envs per policy row). Its co-residency rests on one more
assumption than the plan can check: that the dispatcher spreads a policy workgroup's
4 waves over the CU's 4 SIMDs (two on one SIMD leave 208 VGPRs, below an owner
wave's 320); the abort protocol bounds what a violation costs (an error after ~seconds,
not a hang).

Timeouts. A flag that never comes (~seconds) sets SACENV_STATUS_HANDOFF_TIMEOUT;
from then on every hand-off launch is a no-op on the device (sacenv.h's abort
protocol), ``check()`` raises, and ``run()`` refuses to enqueue more steps once
``check()`` has seen the bit.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import torch

from . import _lib


SIMD_VGPRS = 512       # per lane: the unified architectural + accumulation file of a gfx950 SIMD
VGPR_GRANULE = 8       # allocation granule (wave64)
SIMDS_PER_CU = 4
WAVE_SLOTS = 8         # waves per SIMD
LDS_PER_CU = 160 * 1024


def _alloc(v: int) -> int:
    return -(-int(v) // VGPR_GRANULE) * VGPR_GRANULE


@dataclass(frozen=True)
class CoResidencyPlan:
    cus: int            # compute units of the device
    seg_grid: int       # owner waves (one-wave workgroups, n_pad / 64)
    seg_vgprs: int      # per lane, allocated
    seg_lds: int        # bytes per owner workgroup
    act_grid: int       # policy workgroups (64 rows, 4 waves each)
    act_vgprs: int
    act_lds: int        # bytes per policy workgroup (padded: at most one per CU)
    owner_waves_per_simd: int
    max_envs: int       # the largest env count this pair of kernels admits


def occupancy(params, num_envs: int) -> dict:
    """Both kernels' resources from the library (hipFuncGetAttributes, and
    hipOccupancyMaxActiveBlocksPerMultiprocessor for each alone)."""
    lib = _lib.load()
    v = [C.c_int32() for _ in range(8)]
    _lib.check(lib.sacenv_boat_segment_occupancy(C.byref(params), 0, *[C.byref(x) for x in v[:4]]))
    _lib.check(lib.sacenv_sac_act_occupancy(int(num_envs), *[C.byref(x) for x in v[4:]]))
    k = ("seg_per_cu", "seg_grid", "seg_vgprs", "seg_lds", "act_per_cu", "act_grid", "act_vgprs", "act_lds")
    return {n: x.value for n, x in zip(k, v)}


def make_plan(cus: int, seg_grid: int, seg_vgprs: int, seg_lds: int, act_grid: int, act_vgprs: int,
              act_lds: int, num_envs: int = 0) -> CoResidencyPlan:
    """Per-SIMD VGPR / wave-slot and per-CU LDS accounting (module docstring)."""
    if act_lds * 2 <= LDS_PER_CU:
        raise _lib.SacenvError(f"hand-off policy workgroup LDS {act_lds} B does not exclude a second one per CU")
    sv, av = _alloc(seg_vgprs), _alloc(act_vgprs)
    # owner waves one SIMD can hold next to one policy wave, and the CU's LDS next to one policy workgroup
    per_simd = min((SIMD_VGPRS - av) // sv if sv else WAVE_SLOTS, WAVE_SLOTS - 1)
    if seg_lds:
        per_simd = min(per_simd, (LDS_PER_CU - act_lds) // seg_lds // SIMDS_PER_CU)
    cap = cus * SIMDS_PER_CU * max(per_simd, 0)
    need = -(-seg_grid // (cus * SIMDS_PER_CU))
    if per_simd < 1 or seg_grid > cap:
        raise ValueError(
            f"closed loop cannot be co-resident: {num_envs} envs need {seg_grid} owner waves ({need} per SIMD of "
            f"{cus * SIMDS_PER_CU}, {sv} VGPRs each); with one {av}-VGPR policy wave beside them a SIMD holds "
            f"{max(per_simd, 0)}: use at most {64 * cap} envs per GPU")
    return CoResidencyPlan(cus, seg_grid, sv, seg_lds, act_grid, av, act_lds, need, 64 * cap)


def plan(env, n_cu: int | None = None) -> CoResidencyPlan:
    """The co-residency plan of a closed loop over ``env`` (raises if none exists)."""
    cus = int(n_cu) if n_cu is not None else torch.cuda.get_device_properties(env.device).multi_processor_count
    o = occupancy(env.params, env.num_envs)
    return make_plan(cus, o["seg_grid"], o["seg_vgprs"], o["seg_lds"], o["act_grid"], o["act_vgprs"], o["act_lds"],
                     env.num_envs)


class ClosedLoop:
    """Drives ``env`` (a ``VecBoatEnv``) with ``agent`` (a ``NativeSAC``): ``run`` is the
    eager form unless ``handoff=True`` (module docstring). A context manager: ``close``
    (or leaving the ``with`` block) releases the hand-off's policy queue."""

    def __init__(self, env, agent, segment: int = _lib.REFILL_PERIOD, n_cu: int | None = None,
                 handoff: bool = False):
        if segment < 1 or (env.autoreset and segment > _lib.REFILL_PERIOD):
            raise ValueError(f"segment must be 1..{_lib.REFILL_PERIOD}")
        self.env, self.agent, self.K = env, agent, int(segment)
        self.handoff = bool(handoff)
        self.seq = 0
        self.failed = False
        self._keep = []
        self._policy_handle = None
        self.plan = None
        if not self.handoff:
            return
        self.plan = plan(env, n_cu)
        dev = env.device
        nw = env.n_pad // 64
        self.act_ready = torch.zeros(nw, dtype=torch.int32, device=dev)
        self.step_done = torch.zeros(nw, dtype=torch.int32, device=dev)
        self.actions = torch.zeros((self.K, env.num_envs), dtype=torch.float32, device=dev)
        self.status = env.status[1:2]
        # The two sides must run concurrently. The policy gets a hardware queue of its
        # own (sacenv.h: two ordinary streams may share a queue and serialise, which
        # deadlocks the hand-off); that stream is a BLOCKING one (hipExtStreamCreateWith-
        # CUMask takes no flags), and the legacy null stream -- torch's default --
        # implicitly waits for blocking streams, so the env's persistent launch goes on
        # a non-blocking stream of its own, ordered after the caller's stream by events.
        self.env_stream = torch.cuda.Stream(device=dev)
        h = C.c_void_p()
        with torch.cuda.device(dev):
            _lib.check(_lib.load().sacenv_stream_create_exclusive(C.byref(h)))
        self._policy_handle = h
        self.policy_stream = torch.cuda.ExternalStream(h.value, device=dev)

    def close(self) -> None:
        """Release the policy's hardware queue once its work is done (waits for that
        stream only, not the device)."""
        h = getattr(self, "_policy_handle", None)
        if h is not None and h.value:
            self.policy_stream.synchronize()
            _lib.check(_lib.load().sacenv_stream_destroy(h))
        self._policy_handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

    def __del__(self):  # a fallback for loops never closed: this stream's sync only
        try:
            self.close()
        except Exception:  # noqa: BLE001  (interpreter shutdown)
            pass

    def check(self) -> None:
        """Synchronise and raise if a hand-off timed out (then this loop stays refused)."""
        bits = int(self.status.item())
        if bits & _lib.STATUS_HANDOFF_TIMEOUT:
            self.failed = True
            raise _lib.SacenvError("closed loop: a hand-off timed out (the env or the policy never "
                                   "published); the device refuses further hand-off launches")
        self.env.check_status()

    def run(self, eps: torch.Tensor) -> None:
        """``eps.shape[0]`` (<= segment) steps: policy draws ``eps[k]`` (f32 [N]) for step k,
        in this loop's form (the hand-off with ``handoff=True``, else ``run_eager``)."""
        if self.handoff:
            self.run_handoff(eps)
        else:
            self.run_eager(eps)

    def run_handoff(self, eps: torch.Tensor) -> None:
        """The hand-off form: the policy launches and ONE persistent env launch, handing
        off through the per-wave flags. Enqueues everything; the env's refill
        (autoreset) follows each segment on the env's stream."""
        if not self.handoff:
            raise RuntimeError("construct the ClosedLoop with handoff=True for the hand-off form")
        if self.failed:
            raise _lib.SacenvError("closed loop refused: an earlier hand-off timed out")
        K = int(eps.shape[0])
        if K > self.K or eps.shape[1] != self.env.num_envs:
            raise ValueError(f"eps must be [<= {self.K}, {self.env.num_envs}]")
        env, q0 = self.env, self.seq
        if q0 + K >= 0x7FFFFFFF:
            raise OverflowError("sequence numbers exhausted: build a new ClosedLoop")
        ps, es = self.policy_stream, self.env_stream
        cur = torch.cuda.current_stream(env.device)
        # both sides start after every earlier write on the caller's stream (reset, the
        # previous segment, its refill): the flags order the steps of a segment, the
        # streams the rest
        ps.wait_stream(cur)
        es.wait_stream(cur)
        obs = env.obs
        with torch.cuda.stream(ps):
            for k in range(K):
                self.agent.choose_action_handoff(
                    obs, eps[k], self.actions[k], obs_ready=self.step_done, obs_want=q0 + k,
                    act_ready=self.act_ready, act_value=q0 + k + 1, status=self.status)
        with torch.cuda.stream(es):
            env.segment_async(self.actions, K, act_ready=self.act_ready, step_done=self.step_done, seq0=q0)
        cur.wait_stream(es)  # the caller's stream continues after both sides
        cur.wait_stream(ps)
        self.seq = q0 + K
        self._keep = [eps]

    def run_eager(self, eps: torch.Tensor) -> None:
        """The same ``eps.shape[0]`` steps as ``run`` (the same results, bit for bit), as
        main.py:78-81 orders them: per step one ``choose_action`` launch (at full
        occupancy) then one ``sacenv_boat_step`` launch, both on the caller's stream.
        When the policy dominates the step -- the reference's 256-256 actor on
        65 536 envs: ~76 us against ~5 us -- this beats the hand-off, whose policy
        workgroups run one per CU beside the resident owner waves."""
        if self.failed:
            raise _lib.SacenvError("closed loop refused: an earlier hand-off timed out")
        K = int(eps.shape[0])
        if K > self.K or eps.shape[1] != self.env.num_envs:
            raise ValueError(f"eps must be [<= {self.K}, {self.env.num_envs}]")
        env = self.env
        for k in range(K):
            a = self.agent.choose_action(env.obs, eps=eps[k])
            env.step_async(a.view(-1))
        self._keep = [eps]
