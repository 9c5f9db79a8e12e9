"""Env-instance data parallelism across the GPUs of a node.

Envs are independent (no cross-env term in BoatEnv.step), so each rank owns
a contiguous block of global env ids [rank*N, (rank+1)*N) and seeds every env
by its GLOBAL id: results do not depend on the world size. The only
collective is the all-gather of the packed per-env record that the step
kernel already writes contiguously (VecBoatEnv.record), per step
(``gather_records``) or per segment of steps (``SegmentPool``):

    [ obs f32 N x 11 | reward f32 N | done u8 N | term u8 N ]  = 50 B/env

so the gather needs no packing kernel. Over RCCL (backend "nccl") this is
``all_gather_into_tensor``; gloo (CPU tests) falls back to list all_gather.

The shared replay buffer consumes whole transitions (s, a, r, s', terminal)
(main.py:83-88, agent/buffer.py:13-22). The record alone cannot form them:
for an env that ended (and auto-reset) its obs is already the NEXT episode's
first obs. The pooled row of a step is the transition row the step kernel
writes itself (``sacenv_boat_step_pooled``, ``TransitionLayout``: s' -- the
obs before any reset --, reward, action, term, and in experiment 2 the one obs
entry a fresh Boat does not fix; 53 B per env, 57 in experiment 2);
``TransitionStream`` turns consecutive pooled rows back into (s, a, r, s',
code). ``sacenv.replay.StagedReplay`` samples the pooled replay buffer straight
out of a segment's rows (the exchange that scales).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from ._lib import TRANS_OBS, trans_bytes  # noqa: F401
from .vec_env import RECORD_BYTES


def shard(rank: int, world: int, envs_per_rank: int) -> tuple[int, int]:
    """(env_id_offset, count) of this rank's envs."""
    if not (0 <= rank < world):
        raise ValueError("rank out of range")
    return rank * envs_per_rank, envs_per_rank


@dataclass(frozen=True)
class RecordLayout:
    n: int  # envs per rank

    @property
    def nbytes(self) -> int:
        return RECORD_BYTES * self.n

    def views(self, buf: torch.Tensor):
        """(obs [n,11] f32, reward [n] f32, done [n] u8, term [n] u8) views of one record."""
        n = self.n
        if buf.dtype != torch.uint8 or buf.numel() != self.nbytes:
            raise ValueError("record buffer must be uint8 of 50*n bytes")
        obs = buf[: 44 * n].view(torch.float32).view(n, 11)
        reward = buf[44 * n: 48 * n].view(torch.float32)
        return obs, reward, buf[48 * n: 49 * n], buf[49 * n: 50 * n]

    def pack(self, obs, reward, done, term) -> torch.Tensor:
        buf = torch.empty(self.nbytes, dtype=torch.uint8, device=obs.device)
        o, r, d, t = self.views(buf)
        o.copy_(obs.to(torch.float32))
        r.copy_(reward.to(torch.float32))
        d.copy_(done.to(torch.uint8))
        t.copy_(term.to(torch.uint8))
        return buf

    def unpack_gathered(self, gathered: torch.Tensor, world: int):
        """Global (obs [world*n,11], reward, done, term), in global env-id order."""
        parts = [self.views(gathered[r * self.nbytes:(r + 1) * self.nbytes]) for r in range(world)]
        return tuple(torch.cat([p[i] for p in parts]) for i in range(4))


@dataclass(frozen=True)
class TransitionLayout:
    """One rank's pooled row for one step, as ``sacenv_boat_step_pooled`` writes it
    (per-field arrays of n_pad entries; ``_lib.trans_bytes(experiment)`` per env):

        [ s' f32 [n_pad][11] | reward f32 | action f32 | term u8 | obs3_next f32 (exp 2) ]

    s' is the obs BEFORE any auto-reset (the terminal obs of envs that ended);
    done = term != 0. In experiment 2 the next transition's s of an env that
    ended is the fresh-Boat obs (``first_obs_template``) with entry 3 =
    obs3_next; elsewhere the template itself.
    """
    n: int            # envs per rank
    n_pad: int        # the arena's padded row count (n rounded up to 64)
    experiment: int = 6

    @property
    def per_env(self) -> int:
        return trans_bytes(self.experiment)

    @property
    def nbytes(self) -> int:
        return self.per_env * self.n_pad

    def views(self, row: torch.Tensor):
        """(s' [n, 11], reward [n], action [n], term [n], obs3_next [n] or None)."""
        n, NP, K = self.n, self.n_pad, TRANS_OBS
        if row.dtype != torch.uint8 or row.numel() != self.nbytes:
            raise ValueError("row must be uint8 of TransitionLayout.nbytes")
        f = lambda a, b: row[a * NP: b * NP].view(torch.float32)[:n]  # noqa: E731
        sp = row[: 4 * K * NP].view(torch.float32).view(NP, K)[:n]
        o = 4 * K
        obs3 = f(o + 9, o + 13) if self.experiment == 2 else None
        return sp, f(o, o + 4), f(o + 4, o + 8), row[(o + 8) * NP: (o + 9) * NP][:n], obs3

    def pack(self, s_next, reward, action, obs3_next, term) -> torch.Tensor:
        """Host-side packing (tests, and hosts without the kernel's buffers); s_next is
        the [n, 11] obs."""
        row = torch.zeros(self.nbytes, dtype=torch.uint8, device=s_next.device)
        sp, r, a, t, o3 = self.views(row)
        sp.copy_(s_next[:, :TRANS_OBS].to(torch.float32))
        r.copy_(reward.reshape(r.shape).to(torch.float32))
        a.copy_(action.reshape(a.shape).to(torch.float32))
        t.copy_(term.reshape(t.shape).to(torch.uint8))
        if o3 is not None:
            o3.copy_(obs3_next.reshape(o3.shape).to(torch.float32))
        return row

    def unpack_gathered(self, gathered: torch.Tensor, world: int):
        """Global (s' [world*n, 11], reward, action, term, obs3_next or None) in global env-id order."""
        parts = [self.views(gathered[r * self.nbytes:(r + 1) * self.nbytes]) for r in range(world)]
        cat = lambda i: torch.cat([p[i] for p in parts])  # noqa: E731
        return cat(0), cat(1), cat(2), cat(3), (cat(4) if self.experiment == 2 else None)


class TransitionStream:
    """Pooled rows of consecutive steps -> (s, a, r, s', code) of every global env.

    ``s`` is the obs the action was taken on: the previous step's s', or for an
    env that ended there the first obs of its new episode (``first_obs``, the
    fresh-Boat template, with entry 3 = that row's obs3_next in experiment 2);
    the reset obs for the first step (the stream starts at a reset). ``s'`` is
    the step's obs before any auto-reset, as the row holds it. ``code`` is the
    term code (the replay buffer derives terminal from it, main.py:83-88);
    done = code != 0."""

    def __init__(self, layout: TransitionLayout, world: int, reset_obs: torch.Tensor,
                 first_obs: torch.Tensor):
        self.layout, self.world = layout, int(world)
        self.prev = reset_obs.to(torch.float32).clone()
        dev = self.prev.device
        self.first = first_obs.to(torch.float32).to(dev).reshape(1, -1)

    def push(self, gathered_row: torch.Tensor):
        s_next, reward, action, term, obs3 = self.layout.unpack_gathered(gathered_row, self.world)
        s = self.prev
        done = term != 0
        fresh = self.first.expand_as(s_next).clone()
        if obs3 is not None:
            fresh[:, 3] = obs3
        self.prev = torch.where(done[:, None], fresh, s_next)
        return s, action.clone(), reward.clone(), s_next.clone(), term.clone()


def gather_records(record: torch.Tensor, out: torch.Tensor | None = None, group=None) -> torch.Tensor:
    """All-gather every rank's packed record into one [world * bytes] buffer."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    if out is None:
        out = torch.empty(world * record.numel(), dtype=torch.uint8, device=record.device)
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, record, group=group)
    else:
        chunks = list(out.chunk(world))
        dist.all_gather(chunks, record, group=group)
    return out


class SegmentPool:
    """Pools a segment of steps' records with ONE all-gather.

    Step j of a segment copies the packed record(s) into row j of a staging
    buffer [seg][record_bytes] (graph-capturable: a device copy); ``flush``
    all-gathers the filled rows on a side stream, so the next segment steps
    while xGMI moves this one. Gathered layout: [world][n_steps][record_bytes]
    (``step_records`` slices it back per step). Two staging buffers alternate;
    ``begin`` makes the stepping stream wait for the gather that last used the
    buffer about to be refilled. Fewer, larger collectives than one per step:
    at 65 536 envs a segment of 256 steps is 840 MB per rank.
    """

    def __init__(self, record_bytes: int, seg: int, device, group=None, n_buffers: int = 2):
        import torch.distributed as dist
        self.rb, self.seg, self.group = int(record_bytes), int(seg), group
        self.world = dist.get_world_size(group)
        self.device = torch.device(device)
        self.stage = [torch.empty(self.seg * self.rb, dtype=torch.uint8, device=self.device)
                      for _ in range(n_buffers)]
        self.gathered = [torch.empty(self.world * self.seg * self.rb, dtype=torch.uint8, device=self.device)
                         for _ in range(n_buffers)]
        self.cuda = self.device.type == "cuda"
        self.side = torch.cuda.Stream(device=self.device) if self.cuda else None
        self.done = [None] * n_buffers
        self.buf, self.fill, self.flushes = 0, 0, 0
        self.last = None  # (gathered buffer, n_steps) of the latest flush

    def _cur(self):
        return torch.cuda.current_stream(self.device) if self.cuda else None

    def begin(self) -> None:
        """Before writing row 0 of the current buffer: its previous gather is done."""
        if self.fill == 0 and self.done[self.buf] is not None:
            self._cur().wait_event(self.done[self.buf])

    def row(self, j: int, buf: int | None = None) -> torch.Tensor:
        """Row j of the current (or given) staging buffer, for kernels that write it."""
        b = self.buf if buf is None else buf
        return self.stage[b][j * self.rb:(j + 1) * self.rb]

    def stage_row(self, j: int, records, buf: int | None = None) -> None:
        """Copy one step's packed record(s) (uint8 tensors, concatenated) into row j."""
        b = self.buf if buf is None else buf
        off = j * self.rb
        for r in records:
            n = r.numel()
            self.stage[b][off: off + n].copy_(r)
            off += n
        if off != (j + 1) * self.rb:
            raise ValueError("records do not fill one row")

    def push(self, records) -> None:
        """Stage the next step (eager use); flushes when the segment is full."""
        self.begin()
        self.stage_row(self.fill, records)
        self.fill += 1
        if self.fill == self.seg:
            self.flush()

    def flush(self, n_steps: int | None = None):
        """All-gather the current buffer's first n_steps rows (default: the filled ones)."""
        n = self.fill if n_steps is None else int(n_steps)
        if n == 0:
            return None
        b = self.buf
        src = self.stage[b][: n * self.rb]
        out = self.gathered[b][: self.world * n * self.rb]
        if self.cuda:
            self.side.wait_stream(self._cur())
            with torch.cuda.stream(self.side):
                gather_records(src, out, self.group)
                ev = torch.cuda.Event()
                ev.record(self.side)
            self.done[b] = ev
        else:
            gather_records(src, out, self.group)
        self.buf, self.fill = (b + 1) % len(self.stage), 0
        self.flushes += 1
        self.last = (out, n)
        return out

    def wait(self) -> None:
        """The stepping stream waits for every gather in flight."""
        if self.cuda:
            for ev in self.done:
                if ev is not None:
                    self._cur().wait_event(ev)

    def step_records(self, gathered: torch.Tensor, n_steps: int, k: int) -> torch.Tensor:
        """Step k's pooled record [world * record_bytes], rank order (a copy)."""
        g = gathered.view(self.world, n_steps, self.rb)
        return g[:, k].reshape(-1).clone()


def shard_owner(rows, cntr: int, mem_size: int, period: int, n_per_rank: int):
    """Which rank wrote ring row ``rows`` of a pooled replay buffer that appends
    ``period = world * n_per_rank`` rows per step in global env order (rank r's at
    offset r * n_per_rank): the row holds the latest global sequence number
    s = row (mod mem_size) below ``cntr``; its writer is (s mod period) // n_per_rank.
    The rule ``sacenv_replay_sample_shard`` applies on the device (ShardedReplayBuffer)."""
    import numpy as np
    rows = np.asarray(rows, dtype=np.int64)
    s = rows + mem_size * ((cntr - 1 - rows) // mem_size)
    return (s % period) // n_per_rank


class SegmentExchange:
    """The replay exchange of the persistent segments (StagedReplay), on the stepping
    stream after each segment's refill.

    Measured on the box (round 6, kernel traces, ``tools/prof_staged3.py``): a segment
    launch's owner waves are one per SIMD and bound by their own instruction issue, so a
    kernel co-running with a launch slows the owner waves it shares SIMDs with and the
    launch ends with its slowest wave (300 -> 360-440 us with the pack, the draws or a
    16-workgroup collective stand-in beside it); side kernels co-running with the refill
    slow its latency chain as much (k_need_masks 6 -> 85-95 us, k_refill_fit 28 -> 90-115
    us); and every wait of the stepping stream on another stream's event cost ~20-40 us.
    So the exchange's local work runs on the stepping stream, after refill g (with the
    counter-based draws and the all-gather, ``sampler.fused``: the three as ONE launch,
    ``side_segment``, the unpack then always one segment behind its pack, collective or
    not):

    - the unpack of segment g - 1 (at N > 1: behind its collective, which ran beside
      launch g), the pack of segment g's share (``pack_segment``), at one rank with no
      collective the unpack of segment g at once, and ``prepare(g + 1)``: the
      counter-based draws of segment g + 2, which also mark segment g + 1's rows and
      count segment g + 2's pack tiles;
    - ``coll``: the collective of segment g behind its pack (``collect_segment``: the
      all-gather or the all-reduce; at one rank the stand-in, if any), overlapped with
      launch g + 1 -- the one piece that cannot wait;
    - MT-exact draws (one workgroup walking the MT chain, ~140 us) run on ``sd`` as soon as
      they are enqueued, beside launch g, and launch g + 1 waits for them.

    ``last`` holds the batches of the latest unpacked segment (``wait()`` unpacks one
    still pending). ``sampler`` is a ``sacenv.replay.StagedReplay`` or anything with its
    methods; on the CPU (no streams) everything runs in order. ``check()`` after a timed
    region raises on a segment the sampler flagged invalid."""

    def __init__(self, sampler, device):
        self.sampler = sampler
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        if self.cuda:
            self.sd = torch.cuda.Stream(device=self.device)
            self.coll = torch.cuda.Stream(device=self.device)
        self.mt = getattr(sampler, "sampler", None) == "mt"
        self.fused = bool(getattr(sampler, "fused", False))
        # a collective (or its stand-in) runs between the pack and the unpack
        self.collective = (getattr(sampler, "world", 1) > 1 or getattr(sampler, "standin", None) is not None)
        self.g = 0               # segments exchanged so far
        self.started = False
        self._ready = {}         # segment -> events its launch waits for
        self._pending = None     # (segment, its collective's event): packed, not unpacked yet
        self._launched = None    # (MT-exact draws) the last two launches' end events
        self.exchanges = 0
        self.last = None         # the batches of the latest unpacked segment

    def _cur(self):
        return torch.cuda.current_stream(self.device) if self.cuda else None

    def _record(self, stream):
        ev = torch.cuda.Event()
        ev.record(stream)
        return ev

    def start(self, obs: torch.Tensor) -> None:
        """The obs every env starts from (the s of the first stored transition); the
        first segments' draws and marks, on the stepping stream."""
        self.sampler.begin(obs)
        if self.cuda:
            # the side streams continue the sampling stream begin()'s draws advance on this
            # stream: they must not run ahead of them
            for st in (self.sd, self.coll):
                st.wait_stream(self._cur())
        self.started, self.g, self._pending = True, 0, None

    def stage_args(self) -> dict:
        """The row arguments of the segment about to be stepped."""
        return self.sampler.stage_args(self.g)

    def before(self) -> None:
        """(MT-exact draws) the stepping stream waits for the draws and marks of the
        segment about to be launched."""
        for ev in self._ready.pop(self.g, ()):
            self._cur().wait_event(ev)

    def launched(self) -> None:
        """Right after the segment launch was enqueued (before its refill): the MT-exact
        draws after segment g's launch wait for launch g - 1's end (the buffers they
        rewrite)."""
        if self.cuda and self.mt:
            self._launched = (self._launched or [])[-1:] + [self._record(self._cur())]

    def _unpack_pending(self) -> None:
        g, ev_c = self._pending
        if self.cuda and ev_c is not None:
            self._cur().wait_event(ev_c)
        self.last = self.sampler.unpack_segment(g)
        self._pending = None

    def after(self) -> None:
        g = self.g
        if not self.cuda:
            self.sampler.prepare(g + 1)
            self.last = self.sampler.sample_segment(g)
        elif self.fused:
            pend = self._pending
            if pend is not None and pend[1] is not None:
                self._cur().wait_event(pend[1])
            got = self.sampler.side_segment(g, pend[0] if pend is not None else None)
            if pend is not None:
                self.last = got
            self._pending = (g, None)
            if self.collective:
                packed = self._record(self._cur())
                with torch.cuda.stream(self.coll):
                    self.coll.wait_event(packed)
                    self.sampler.collect_segment(g)
                    self._pending = (g, self._record(self.coll))
        else:
            if self._pending is not None:
                self._unpack_pending()
            self.sampler.pack_segment(g)
            if self.collective:
                packed = self._record(self._cur())
                with torch.cuda.stream(self.coll):
                    self.coll.wait_event(packed)
                    self.sampler.collect_segment(g)
                    self._pending = (g, self._record(self.coll))
            else:
                self.last = self.sampler.unpack_segment(g)
            if self.mt:  # beside launch g (after launch g - 1's end); launch g + 1 waits for it
                with torch.cuda.stream(self.sd):
                    if self._launched and len(self._launched) == 2:
                        self.sd.wait_event(self._launched[0])
                    self.sampler.prepare(g + 1)
                    self._ready[g + 1] = [self._record(self.sd)]
            else:
                self.sampler.prepare(g + 1)
        self.g += 1
        self.exchanges += 1

    def wait(self) -> None:
        """Unpack the segment still pending; the stepping stream waits for every exchange
        in flight."""
        if self.cuda:
            if self._pending is not None:
                self._unpack_pending()
            for st in (self.sd, self.coll):
                self._cur().wait_stream(st)
        self._ready.clear()

    def check(self) -> None:
        """Raise if the sampler reported an invalid segment (a poisoned MT stream, an
        overflowed all-gather chunk). Synchronises: call it outside a timed region."""
        chk = getattr(self.sampler, "check", None)
        if chk is not None:
            chk()
