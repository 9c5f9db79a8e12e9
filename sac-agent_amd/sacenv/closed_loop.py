"""The acting loop of main.py:70-91 -- ``choose_action`` then ``env.step`` -- as two
device-side pipelines handing off through per-owner-wave flags.

The env runs as persistent segment launches (``VecBoatEnv.segment_async``,
``sacenv_boat_segment``: up to 128 steps per launch, the carried state in
registers), the policy as one ``NativeSAC.choose_action_handoff`` launch per step
on a second stream. For owner wave w (64 envs) and sequence number q:

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
bit (tests/test_closed_loop_gpu.py).
"""
from __future__ import annotations

import torch

from . import _lib


class ClosedLoop:
    """Drives ``env`` (a ``VecBoatEnv``) with ``agent`` (a ``NativeSAC``)."""

    def __init__(self, env, agent, segment: int = _lib.REFILL_PERIOD):
        if segment < 1 or (env.autoreset and segment > _lib.REFILL_PERIOD):
            raise ValueError(f"segment must be 1..{_lib.REFILL_PERIOD}")
        self.env, self.agent, self.K = env, agent, int(segment)
        dev = env.device
        nw = env.n_pad // 64
        self.act_ready = torch.zeros(nw, dtype=torch.int32, device=dev)
        self.step_done = torch.zeros(nw, dtype=torch.int32, device=dev)
        self.actions = torch.zeros((self.K, env.num_envs), dtype=torch.float32, device=dev)
        self.status = env.status[1:2]
        self.policy_stream = torch.cuda.Stream(device=dev)
        self.seq = 0
        self._keep = []

    def run(self, eps: torch.Tensor) -> None:
        """``eps.shape[0]`` (<= segment) steps: policy draws ``eps[k]`` (f32 [N]) for step k.
        Enqueues everything; the env's refill (autoreset) follows each segment on the
        env's stream."""
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
        with torch.cuda.stream(ps):
            for k in range(K):
                self.agent.choose_action_handoff(
                    env.obs, eps[k], self.actions[k], obs_ready=self.step_done, obs_want=q0 + k,
                    act_ready=self.act_ready, act_value=q0 + k + 1, status=self.status)
        env.segment_async(self.actions, K, act_ready=self.act_ready, step_done=self.step_done, seq0=q0)
        torch.cuda.current_stream(env.device).wait_stream(ps)  # the policy's launches are done too
        self.seq = q0 + K
        self._keep = [eps]
