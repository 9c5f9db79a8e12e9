"""The acting loop of main.py:70-91 -- ``choose_action`` then ``env.step`` -- as two
device-side pipelines handing off through per-owner-wave flags.

The env runs as persistent segment launches (``VecBoatEnv.segment_async``,
``sacenv_boat_segment``: up to 128 steps per launch, the carried state in
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
workgroup waits for its own owner wave, and an owner wave that is not yet
dispatched would wait for the slots the spinning workgroups hold. ``plan``
(from ``hipOccupancyMaxActiveBlocksPerMultiprocessor`` of both kernels, through
the C ABI) therefore requires the segment grid's even share per CU plus one
policy launch's share per CU to fit in one CU's resources (as fractions of each
kernel's own per-CU limit, which bounds every resource at once), and splits the
policy's rows into launches of at most ``plan.chunk_waves`` owner waves (one
launch per chunk per step, in order on the policy stream: a chunk's workgroups
wait only for owner waves that are already resident). A configuration in which
the segment grid alone does not leave room for one policy workgroup per CU is
refused.

Timeouts. A flag that never comes (~seconds) sets SACENV_STATUS_HANDOFF_TIMEOUT;
from then on every hand-off launch is a no-op on the device (sacenv.h's abort
protocol), ``check()`` raises, and ``run()`` refuses to enqueue more steps once
``check()`` has seen the bit.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass

import torch

from . import _lib


@dataclass(frozen=True)
class CoResidencyPlan:
    cus: int                 # compute units of the device
    seg_blocks_per_cu: int   # segment kernel: resident one-wave workgroups per CU
    seg_grid: int            # owner waves (n_pad / 64)
    act_blocks_per_cu: int   # act kernel: resident 256-thread workgroups per CU
    act_grid: int            # policy workgroups for all rows (64 rows each)
    chunk_waves: int         # owner waves per policy launch

    @property
    def seg_frac(self) -> float:
        """The segment grid's even share of one CU, as a fraction of its per-CU limit."""
        return math.ceil(self.seg_grid / self.cus) / self.seg_blocks_per_cu

    @property
    def chunks(self) -> int:
        return -(-self.act_grid // self.chunk_waves)


def occupancy(params, num_envs: int) -> tuple[int, int, int, int]:
    """(segment workgroups per CU, segment grid, act workgroups per CU, act grid) from the
    library (hipOccupancyMaxActiveBlocksPerMultiprocessor of the launches' kernels)."""
    lib = _lib.load()
    bs, gs, ba, ga = C.c_int32(), C.c_int32(), C.c_int32(), C.c_int32()
    _lib.check(lib.sacenv_boat_segment_occupancy(C.byref(params), 0, C.byref(bs), C.byref(gs)))
    _lib.check(lib.sacenv_sac_act_occupancy(int(num_envs), C.byref(ba), C.byref(ga)))
    return bs.value, gs.value, ba.value, ga.value


def make_plan(cus: int, seg_per_cu: int, seg_grid: int, act_per_cu: int, act_grid: int,
              num_envs: int = 0) -> CoResidencyPlan:
    """The largest policy chunk whose even share per CU fits beside the segment grid's."""
    if seg_per_cu < 1 or act_per_cu < 1:
        raise _lib.SacenvError(f"occupancy query returned {seg_per_cu} / {act_per_cu} workgroups per CU")
    seg_frac = math.ceil(seg_grid / cus) / seg_per_cu
    per_cu = math.floor((1.0 - seg_frac) * act_per_cu + 1e-9)   # policy workgroups per CU beside it
    if per_cu < 1:
        raise ValueError(
            f"closed loop cannot be co-resident: {num_envs} envs need {seg_grid} owner waves "
            f"({math.ceil(seg_grid / cus)} per CU of {cus}, limit {seg_per_cu}), leaving no room for a "
            f"policy workgroup (limit {act_per_cu} per CU); use fewer envs per GPU")
    return CoResidencyPlan(cus, seg_per_cu, seg_grid, act_per_cu, act_grid, min(act_grid, per_cu * cus))


def max_envs(cus: int, seg_per_cu: int, act_per_cu: int) -> int:
    """The largest env count (a multiple of 64) ``make_plan`` accepts."""
    waves_per_cu = math.floor(seg_per_cu * (1.0 - 1.0 / act_per_cu) + 1e-9)
    return 64 * cus * waves_per_cu


def plan(env, n_cu: int | None = None) -> CoResidencyPlan:
    """The co-residency plan of a closed loop over ``env`` (raises if none exists)."""
    cus = int(n_cu) if n_cu is not None else torch.cuda.get_device_properties(env.device).multi_processor_count
    bs, gs, ba, ga = occupancy(env.params, env.num_envs)
    return make_plan(cus, bs, gs, ba, ga, env.num_envs)


class ClosedLoop:
    """Drives ``env`` (a ``VecBoatEnv``) with ``agent`` (a ``NativeSAC``)."""

    def __init__(self, env, agent, segment: int = _lib.REFILL_PERIOD, n_cu: int | None = None):
        if segment < 1 or (env.autoreset and segment > _lib.REFILL_PERIOD):
            raise ValueError(f"segment must be 1..{_lib.REFILL_PERIOD}")
        self.env, self.agent, self.K = env, agent, int(segment)
        self.plan = plan(env, n_cu)
        dev = env.device
        nw = env.n_pad // 64
        self.act_ready = torch.zeros(nw, dtype=torch.int32, device=dev)
        self.step_done = torch.zeros(nw, dtype=torch.int32, device=dev)
        self.actions = torch.zeros((self.K, env.num_envs), dtype=torch.float32, device=dev)
        self.status = env.status[1:2]
        self.policy_stream = torch.cuda.Stream(device=dev)
        self.seq = 0
        self.failed = False
        self._keep = []
        # the policy launches of one step: (row range, flag range) per chunk
        cw, N = self.plan.chunk_waves, env.num_envs
        self.chunks = [(64 * c0, min(N, 64 * (c0 + cw)), c0, min(nw, c0 + cw))
                       for c0 in range(0, self.plan.act_grid, cw)]

    def check(self) -> None:
        """Synchronise and raise if a hand-off timed out (then this loop stays refused)."""
        bits = int(self.status.item())
        if bits & _lib.STATUS_HANDOFF_TIMEOUT:
            self.failed = True
            raise _lib.SacenvError("closed loop: a hand-off timed out (the env or the policy never "
                                   "published); the device refuses further hand-off launches")
        self.env.check_status()

    def run(self, eps: torch.Tensor) -> None:
        """``eps.shape[0]`` (<= segment) steps: policy draws ``eps[k]`` (f32 [N]) for step k.
        Enqueues everything; the env's refill (autoreset) follows each segment on the
        env's stream."""
        if self.failed:
            raise _lib.SacenvError("closed loop refused: an earlier hand-off timed out")
        K = int(eps.shape[0])
        if K > self.K or eps.shape[1] != self.env.num_envs:
            raise ValueError(f"eps must be [<= {self.K}, {self.env.num_envs}]")
        env, q0 = self.env, self.seq
        if q0 + K >= 0x7FFFFFFF:
            raise OverflowError("sequence numbers exhausted: build a new ClosedLoop")
        ps = self.policy_stream
        # the policy's first read (row q0: step_done >= q0 holds at once) must follow
        # every earlier write of the obs on the env's stream (reset, the previous
        # segment): the flags order the steps of a segment, the stream the rest
        ps.wait_stream(torch.cuda.current_stream(env.device))
        obs = env.obs
        with torch.cuda.stream(ps):
            for k in range(K):
                for r0, r1, c0, c1 in self.chunks:
                    self.agent.choose_action_handoff(
                        obs[r0:r1], eps[k, r0:r1], self.actions[k, r0:r1],
                        obs_ready=self.step_done[c0:c1], obs_want=q0 + k,
                        act_ready=self.act_ready[c0:c1], act_value=q0 + k + 1, status=self.status)
        env.segment_async(self.actions, K, act_ready=self.act_ready, step_done=self.step_done, seq0=q0)
        torch.cuda.current_stream(env.device).wait_stream(ps)  # the policy's launches are done too
        self.seq = q0 + K
        self._keep = [eps]
