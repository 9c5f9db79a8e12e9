"""Device replay buffer: agent/buffer.py:3-35 on the GPU.

Two front ends over one C-ABI arena (libsacenv.so, gfx950):

* ``DeviceReplayBuffer``: batched and device-resident. ``store_batch`` appends
  the transitions of all envs of a step (one launch). ``store_env_step`` takes a
  ``VecBoatEnv`` step directly: the new_state of an env that auto-reset is its
  terminal obs (``info['final_obs']``), and terminal = the env's last
  termination is reached_goal (main.py:83-88, with the info dict's persistence). ``sample`` returns device tensors. Sampling follows
  ``np.random.choice`` on the buffer's own MT19937 stream, seeded like
  ``np.random.seed(seed)``.
* ``ReplayBuffer``: the drop-in for ``agent.buffer.ReplayBuffer``. It has the
  same constructor, ``store_transition`` and ``sample_buffer`` (numpy in,
  numpy out), and samples from numpy's GLOBAL RNG stream: the state is
  uploaded, drawn on the GPU and written back, so the batches equal the
  reference's for the same ``np.random`` state.

There is no CPU path: without libsacenv.so these classes raise.
"""
from __future__ import annotations

import ctypes as C
import weakref

import numpy as np
import torch

from . import _lib

TERMINAL_GOAL = 1 << 1   # terminal = (code == 1): env term reached_goal, or a 0/1 done array


class DeviceReplayBuffer:
    def __init__(self, max_size: int, input_shape, n_actions: int, *, device=None, seed: int = 0,
                 reward_f32: bool = True, terminal_mask: int = TERMINAL_GOAL):
        self.lib = _lib.load()
        self.device = torch.device(device if device is not None else "cuda")
        if self.device.type != "cuda":
            raise RuntimeError("DeviceReplayBuffer runs on a GPU (HIP); no CPU path")
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        shape = (int(input_shape),) if np.isscalar(input_shape) else tuple(int(d) for d in input_shape)
        self.input_shape = shape
        self.mem_size = int(max_size)
        self.n_actions = int(n_actions)
        p = _lib.ReplayParams()
        p.mem_size, p.obs_dim, p.act_dim = self.mem_size, int(np.prod(shape)), self.n_actions
        p.reward_f32, p.terminal_mask = int(bool(reward_f32)), int(terminal_mask)
        self.params = p
        self._pp = C.byref(p)
        self.layout = L = _lib.replay_layout(p)
        self.arena = torch.zeros(int(L.total_bytes), dtype=torch.uint8, device=self.device)
        M, D, A = self.mem_size, p.obs_dim, self.n_actions

        def view(off, dtype, *shp):
            esz = torch.empty((), dtype=dtype).element_size()
            return self.arena[off: off + int(np.prod(shp)) * esz].view(dtype).view(*shp)

        self.state_memory = view(L.state, torch.float32, M, *shape)
        self.new_state_memory = view(L.new_state, torch.float32, M, *shape)
        self.action_memory = view(L.action, torch.float32, M, A)
        self.reward_memory = view(L.reward, torch.float64, M)
        self.terminal_memory = view(L.terminal, torch.uint8, M)
        self._cntr = view(L.mem_cntr, torch.int64, 1)
        self.mt_key = view(L.mt_key, torch.int32, _lib.MT_N)
        self.mt_pos = view(L.mt_pos, torch.int32, 1)
        self.mem_cntr = 0                        # host mirror (buffer.py:6)
        # env -> u8 [num_envs] info['termination'] codes; weak keys: an env that is
        # garbage-collected takes its bytes with it (no id() reuse by a new env)
        self._last_term = weakref.WeakKeyDictionary()
        _lib.check(self.lib.sacenv_replay_init(self._pp, self.arena.data_ptr(), int(seed) & 0xFFFFFFFF,
                                               self.stream))

    @property
    def stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    def _dev(self, x, dtype):
        t = torch.as_tensor(x, device=self.device)
        return t.to(dtype).contiguous() if t.dtype != dtype else t.contiguous()

    def store_batch(self, state, action, reward, new_state, code, final_state=None,
                    last_term=None, graph_safe: bool = False) -> None:
        """Append n transitions (rows in order, buffer.py:13-22). ``code`` is u8:
        terminal = (terminal_mask >> code) & 1; rows with code != 0 take new_state
        from ``final_state`` if it is given. ``last_term`` (u8 [n] device tensor, in/out):
        row i's terminal follows env i's persistent last termination instead
        (``sacenv_replay_store_env``; see ``store_env_step``). By default the host's
        count goes into the launch (one launch, ``sacenv_replay_store_env_at``), which a
        captured graph would freeze; ``graph_safe=True`` reads and advances the device
        count instead (``sacenv_replay_store_env``: a store and an advance launch)."""
        s = self._dev(state, torch.float32)
        n = s.shape[0]
        a = self._dev(action, torch.float32).reshape(n, -1)
        r = self._dev(reward, torch.float32 if self.params.reward_f32 else torch.float64).reshape(n)
        ns = self._dev(new_state, torch.float32)
        c = self._dev(code, torch.uint8).reshape(n)
        fs = None if final_state is None else self._dev(final_state, torch.float32)
        if a.shape[1] != self.n_actions or s.shape != ns.shape:
            raise ValueError("transition shapes do not match the buffer")
        lt = None
        if last_term is not None:
            lt = last_term
            if (lt.dtype != torch.uint8 or lt.device != self.device or lt.numel() != n
                    or not lt.is_contiguous()):
                raise ValueError("last_term must be a contiguous u8 device tensor with one byte per row")
        if graph_safe:  # the device count, read and advanced on the device
            _lib.check(self.lib.sacenv_replay_store_env(
                self._pp, self.arena.data_ptr(), n, s.data_ptr(), a.data_ptr(), r.data_ptr(), ns.data_ptr(),
                None if fs is None else fs.data_ptr(), c.data_ptr(), None if lt is None else lt.data_ptr(),
                self.stream))
        else:  # the host issues every store, so it knows the count: one launch (sacenv.h)
            _lib.check(self.lib.sacenv_replay_store_env_at(
                self._pp, self.arena.data_ptr(), self.mem_cntr, n, s.data_ptr(), a.data_ptr(), r.data_ptr(),
                ns.data_ptr(), None if fs is None else fs.data_ptr(), c.data_ptr(),
                None if lt is None else lt.data_ptr(), self.stream))
        self._keep = (s, a, r, ns, c, fs)
        self.mem_cntr += n

    def store_env_step(self, prev_obs, actions, env, reference_terminal: bool = True) -> None:
        """The transitions of one ``VecBoatEnv.step``: (prev_obs, actions, reward,
        obs or final_obs for envs that ended, terminal).

        ``reference_terminal`` (default, parity with main.py:83-88): terminal is
        ``info['termination'] == 'reached_goal'``, where ``info['termination']``
        is the env's LAST termination -- the reference's info dict keeps it
        across steps and resets (boat_env.py:24-32,120-126), so after a goal
        episode every transition is stored terminal until another ending
        overwrites it. The buffer keeps that byte per env. ``False``: terminal
        only on the step that reached the goal (the evident intent)."""
        last = None
        if reference_terminal:
            last = self._last_term.get(env)
            if last is None or last.numel() != env.num_envs:
                last = torch.zeros(env.num_envs, dtype=torch.uint8, device=self.device)
                self._last_term[env] = last
        self.store_batch(prev_obs, actions, env.reward, env.obs, env.term, final_state=env.final_obs,
                         last_term=last)

    def sample(self, batch_size: int, as_bool: bool = True):
        """sample_buffer (buffer.py:24-35) on device: (states, actions, rewards, states_, dones, idx).
        ``as_bool=False``: dones as the kernel writes them (u8 0/1), with no conversion launch
        (the agent's learn() reads u8)."""
        B = int(batch_size)
        if self.mem_cntr == 0 and B > 0:
            raise ValueError("a must be greater than 0 unless no samples are taken")
        idx = torch.empty(B, dtype=torch.int64, device=self.device)
        st = torch.empty((B, *self.input_shape), dtype=torch.float32, device=self.device)
        ns = torch.empty_like(st)
        ac = torch.empty((B, self.n_actions), dtype=torch.float32, device=self.device)
        rw = torch.empty(B, dtype=torch.float64, device=self.device)
        tm = torch.empty(B, dtype=torch.uint8, device=self.device)
        _lib.check(self.lib.sacenv_replay_sample(
            self._pp, self.arena.data_ptr(), B, self.mem_cntr, idx.data_ptr(), st.data_ptr(),
            ac.data_ptr(), rw.data_ptr(), ns.data_ptr(), tm.data_ptr(), self.stream))
        return st, ac, rw, ns, (tm.bool() if as_bool else tm), idx

    def gather(self, idx: torch.Tensor, as_bool: bool = True):
        """The rows at the given ring indices (buffer.py:28-33 without the draw):
        (states, actions, rewards f64, states_, dones); an index outside the ring gives
        zeros (``sacenv_replay_gather``)."""
        idx = idx.to(device=self.device, dtype=torch.int64).contiguous().reshape(-1)
        B = idx.numel()
        st = torch.empty((B, *self.input_shape), dtype=torch.float32, device=self.device)
        ns = torch.empty_like(st)
        ac = torch.empty((B, self.n_actions), dtype=torch.float32, device=self.device)
        rw = torch.empty(B, dtype=torch.float64, device=self.device)
        tm = torch.empty(B, dtype=torch.uint8, device=self.device)
        _lib.check(self.lib.sacenv_replay_gather(
            self._pp, self.arena.data_ptr(), B, idx.data_ptr(), st.data_ptr(), ac.data_ptr(), rw.data_ptr(),
            ns.data_ptr(), tm.data_ptr(), self.stream))
        return st, ac, rw, ns, (tm.bool() if as_bool else tm)


class ShardedReplayBuffer(DeviceReplayBuffer):
    """The replay buffer pooled over ``world`` ranks (main.py:81-88 with every rank's
    envs feeding one agent/buffer.py:3-35 ring) WITHOUT moving the
    transitions: each rank writes only its own envs' rows, at the ring positions
    the pooled buffer gives them (``sacenv_replay_store_shard``: per step the pooled
    ring appends ``world * n`` rows in global env order, rank r's at offset r*n), and
    ``sample`` draws the pooled buffer's indices on every rank (same seed, same
    stream: ``np.random.choice(max_mem, batch)``) and assembles the batch with one
    integer SUM all-reduce of the gathered bits (each row comes from the one rank
    that wrote it, the others contribute zero bits): the batch equals the pooled
    buffer's bit for bit, and B rows cross the links per ``learn()`` instead of
    every transition of every step (tests/test_dist_cpu.py)."""

    def __init__(self, max_size, input_shape, n_actions, *, rank: int, world: int, envs_per_rank: int,
                 device=None, seed: int = 0, group=None, **kw):
        super().__init__(max_size, input_shape, n_actions, device=device, seed=seed, **kw)
        self.rank, self.world, self.n = int(rank), int(world), int(envs_per_rank)
        self.period, self.offset = self.world * self.n, self.rank * self.n
        if self.period > self.mem_size:
            raise ValueError("one step's pooled rows must fit the ring (world * envs <= max_size)")
        self.group = group

    def store_batch(self, state, action, reward, new_state, code, final_state=None, last_term=None) -> None:
        """This rank's n rows of one pooled step (rank-local inputs, as DeviceReplayBuffer)."""
        s = self._dev(state, torch.float32)
        n = s.shape[0]
        if n != self.n:
            raise ValueError(f"a step stores this rank's {self.n} rows")
        a = self._dev(action, torch.float32).reshape(n, -1)
        r = self._dev(reward, torch.float32 if self.params.reward_f32 else torch.float64).reshape(n)
        ns = self._dev(new_state, torch.float32)
        c = self._dev(code, torch.uint8).reshape(n)
        fs = None if final_state is None else self._dev(final_state, torch.float32)
        _lib.check(self.lib.sacenv_replay_store_shard(
            self._pp, self.arena.data_ptr(), n, self.offset, self.period, s.data_ptr(), a.data_ptr(),
            r.data_ptr(), ns.data_ptr(), None if fs is None else fs.data_ptr(), c.data_ptr(),
            None if last_term is None else last_term.data_ptr(), self.stream))
        self._keep = (s, a, r, ns, c, fs)
        self.mem_cntr += self.period

    def sample(self, batch_size: int, as_bool: bool = True):
        """The pooled buffer's sample_buffer (buffer.py:24-35), identical on every rank
        (``as_bool=False``: dones as u8, as DeviceReplayBuffer.sample)."""
        st, ac, rw, ns, tm, idx = self.sample_many(batch_size, 1)[0]
        return st, ac, rw, ns, (tm if as_bool else tm.to(torch.uint8)), idx

    def sample_many(self, batch_size: int, n_batches: int):
        """``n_batches`` consecutive sample_buffer calls with NO stores between them,
        assembled with ONE SUM all-reduce: the same batches, in the same order, as
        ``n_batches`` ``sample`` calls at this mem_cntr (the index draws continue the
        buffer's one MT19937 stream), for one collective's latency instead of
        ``n_batches``. (The reference's loop stores a step's rows before each learn();
        ``StagedReplay`` samples a segment's learns with the buffer each of them saw.)"""
        import torch.distributed as dist
        B, n = int(batch_size), int(n_batches)
        if n < 1:
            raise ValueError("n_batches must be positive")
        if self.mem_cntr == 0 and B > 0:
            raise ValueError("a must be greater than 0 unless no samples are taken")
        D, A = int(np.prod(self.input_shape)), self.n_actions
        words, views = _packed_batches(B, n, D, A, self.input_shape, self.device)
        tm = torch.empty(B, dtype=torch.uint8, device=self.device)
        for st, ac, rw, ns, tm32, idx in views:
            _lib.check(self.lib.sacenv_replay_sample_shard(
                self._pp, self.arena.data_ptr(), B, self.mem_cntr, self.offset, self.n, self.period,
                idx.data_ptr(), st.data_ptr(), ac.data_ptr(), rw.data_ptr(), ns.data_ptr(), tm.data_ptr(),
                self.stream))
            tm32.copy_(tm.to(torch.int32))
        if self.world > 1:
            dist.all_reduce(words, op=dist.ReduceOp.SUM, group=self.group)
        return [(st, ac, rw, ns, tm32.to(torch.bool), idx) for st, ac, rw, ns, tm32, idx in views]


def _packed_batches(B: int, n: int, D: int, A: int, shape, device):
    """n batches packed as 32-bit words, per batch: reward (f64 = 2 words, first:
    8-B aligned), state, new_state, action (f32), terminal (one word per row);
    each block padded to an even word count. Returns (words, [(st, ac, rw, ns,
    tm32, idx)] views)."""
    per = B * (2 * D + A + 3)
    per += per & 1
    words = torch.zeros(n * per, dtype=torch.int32, device=device)
    views = []
    for i in range(n):
        w = words[i * per: (i + 1) * per]
        rw = w[: 2 * B].view(torch.float64)
        o = 2 * B
        st = w[o: o + B * D].view(torch.float32).view(B, *shape)
        o += B * D
        ns = w[o: o + B * D].view(torch.float32).view(B, *shape)
        o += B * D
        ac = w[o: o + B * A].view(torch.float32).view(B, A)
        o += B * A
        tm32 = w[o: o + B]
        idx = torch.empty(B, dtype=torch.int64, device=device)
        views.append((st, ac, rw, ns, tm32, idx))
    return words, views


class StagedReplay:
    """The pooled replay buffer of main.py:78-90 -- every rank's envs storing one
    transition each per step into ONE agent/buffer.py ring (``ReplayBuffer(mem_size)``,
    buffer.py:13-22) and one ``learn()`` sampling it after every step (buffer.py:24-35)
    -- served from the rows the persistent step launch writes, with no ring and no
    store of rows nobody reads.

    The batches' indices depend only on the sampling stream (np.random.choice on an
    MT19937 state seeded like ``np.random.seed(seed)``) and on how many rows were
    stored before each learn, so they are drawn AHEAD: ``prepare(g)`` draws segment
    g+1's learns and marks the rows of segment g that the learns of segments g and
    g+1 will read (``sacenv_replay_stage_draw`` / ``_stage_mark``); segment g's launch
    (``sacenv_boat_segment`` with ``**stage_args(g)``) writes exactly those rows (64 B
    each); ``sample_segment(g)`` gathers this rank's share of segment g's batches from
    segments g and g-1 (``sacenv_replay_sample_staged``) and, with world > 1, ONE SUM
    all-reduce of the packed batches makes them the pooled buffer's batches, bit for
    bit, on every rank (tests/test_staged_replay_gpu.py). ~27 MB cross the links per
    256-step segment at batch 1 024, whatever the world size.

    Order per segment g (``begin`` did draws 0 and 1 and the marks of segment 0):
    ``stage_args(g)`` -> the launch -> ``prepare(g + 1)`` -> ``sample_segment(g)``. Buffers: the staged rows of segment g are read by
    ``sample_segment(g)`` and ``(g + 1)``, so the launch of segment g + 2 (3 buffers)
    must follow ``sample_segment(g)`` in stream order; a launch consumes (clears) its
    marks (``sacenv.dist.SegmentExchange`` arranges the streams).

    ``sampler``: ``"mt"`` (default) draws every learn from the buffer's one MT19937
    stream exactly as the reference's ``np.random.choice`` would (the parity mode:
    the batches equal a DeviceReplayBuffer's bit for bit); ``"philox"`` draws the
    same distribution -- uniform with replacement over the rows stored, the same
    skip rule -- from a counter-based generator (Philox4x64-10 keyed by the seed,
    counted by (draw, learn)), so a segment's draws are one parallel launch that
    also marks the rows (``sacenv_replay_stage_draw_ctr``; oracle/ctr_sampler.py).
    ``exchange``: ``"allreduce"`` (default) assembles the batches with one SUM
    all-reduce of the 1/world-dense packed batches; ``"allgather"`` packs each
    rank's own rows (100-B records with their slot) into a fixed chunk and
    all-gathers the chunks (about half the bytes per rank of the ring all-reduce),
    then unpacks them into the same words on every rank. Both are bit-exact.
    ``standin`` (world 1 only; bench.py's replay path): a dict(bytes, workgroups, us)
    -- a copy kernel of that many bytes on that many workgroups, resident for that
    long, between the pack and the unpack: the collective's kernel stood in for."""

    N_BUFFERS = 3

    def __init__(self, n: int, n_pad: int, experiment: int, first_obs, *, rank: int = 0, world: int = 1,
                 mem_size: int = 1_000_000, batch: int = 1024, seg: int = 256, seed: int = 0,
                 device=None, group=None, terminal_mask: int = TERMINAL_GOAL, sampler: str = "mt",
                 exchange: str = "allreduce", standin: dict | None = None):
        self.lib = _lib.load()
        self.device = torch.device(device if device is not None else "cuda")
        if self.device.type != "cuda":
            raise RuntimeError("StagedReplay runs on a GPU (HIP); no CPU path")
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        if sampler not in ("mt", "philox") or exchange not in ("allreduce", "allgather"):
            raise ValueError("sampler is 'mt' or 'philox'; exchange is 'allreduce' or 'allgather'")
        self.sampler, self.exchange = sampler, exchange
        self.n, self.n_pad, self.seg, self.batch = int(n), int(n_pad), int(seg), int(batch)
        if not 1 <= self.seg <= _lib.REFILL_PERIOD:
            # the segment launch stages one mark word per step in LDS (REFILL_PERIOD of them)
            raise ValueError(f"seg must be in [1, {_lib.REFILL_PERIOD}]")
        self.rank, self.world, self.group = int(rank), int(world), group
        if standin is not None and group is not None:
            raise ValueError("the collective stand-in is a one-GPU measurement (no process group)")
        # world > 1 with the stand-in and no group: ONE GPU as rank `rank` of a world-rank
        # pooled buffer (bench.py's replay_path_rank_of_W): the collective stood in for, the
        # other ranks' chunks packed once from this GPU's rows under their env ids
        self.emulated = standin is not None and self.world > 1
        if self.emulated and (exchange != "allgather" or sampler != "philox"):
            raise ValueError("the emulated rank runs the counter-based all-gather exchange")
        self.mem_size = int(mem_size)
        self.seed = int(seed)
        sp = _lib.StagedParams()
        sp.period, sp.offset = self.world * self.n, self.rank * self.n
        sp.n, sp.n_pad, sp.seg, sp.experiment = self.n, self.n_pad, self.seg, int(experiment)
        fo = np.asarray(first_obs.cpu() if isinstance(first_obs, torch.Tensor) else first_obs,
                        np.float32).reshape(_lib.OBS_DIM)
        for k in range(_lib.OBS_DIM):
            sp.first_obs[k] = float(fo[k])
        if self.mem_size > self.seg * sp.period:
            raise ValueError(f"mem_size {self.mem_size} > seg * period = {self.seg * sp.period}: a learn could "
                             "reach rows older than the previous segment")
        self.sp, self._spp = sp, C.byref(sp)
        self.period = int(sp.period)
        if sampler == "mt":
            # the sampling stream lives in a replay arena (its key / pos fields)
            self._rb = DeviceReplayBuffer(self.mem_size, (_lib.OBS_DIM,), 1, device=self.device, seed=seed,
                                          reward_f32=True, terminal_mask=terminal_mask)
            self._pp = self._rb._pp
        else:  # (no stream: only the buffer's shape)
            self._rb = None
            p = _lib.ReplayParams()
            p.mem_size, p.obs_dim, p.act_dim = self.mem_size, _lib.OBS_DIM, 1
            p.reward_f32, p.terminal_mask = 1, int(terminal_mask)
            self._params = p
            self._pp = C.byref(p)
        self._status = torch.zeros(4, dtype=torch.int32, device=self.device)
        nb = self.N_BUFFERS
        self.stage = [torch.zeros(self.seg * self.n_pad * 64, dtype=torch.uint8, device=self.device)
                      for _ in range(nb)]
        # env-major (sacenv_boat_segment): env e's row of step j at (e * seg + j) * 64, its mark
        # bit j % 64 in word e * ceil(seg / 64) + j // 64
        self.marks = [torch.zeros(self.n_pad * -(-self.seg // 64), dtype=torch.int64, device=self.device)
                      for _ in range(nb)]
        self._idx = [torch.empty(self.seg * self.batch, dtype=torch.int64, device=self.device) for _ in range(4)]
        self._words = [_packed_batches(self.batch, self.seg, _lib.OBS_DIM, 1, (_lib.OBS_DIM,), self.device)
                       for _ in range(2)]
        # the per-learn views of each (words, idx) buffer pair, built once instead of
        # 256 idx slices per segment (host time the persistent launches do not wait for)
        B = self.batch
        self._batches = {}
        for wi, (_, views) in enumerate(self._words):
            for ii, idx in enumerate(self._idx):
                self._batches[wi, ii] = [(st, ac, rw, ns, tm32, idx[i * B: (i + 1) * B])
                                         for i, (st, ac, rw, ns, tm32, _) in enumerate(views)]
        if sampler == "mt":
            nbytes = C.c_int64()
            _lib.check(self.lib.sacenv_replay_stage_scratch_bytes(self._pp, self.batch, self.seg, C.byref(nbytes)))
            self._scratch = torch.empty(int(nbytes.value), dtype=torch.uint8, device=self.device)
        if exchange == "allgather":
            self.cap, self.chunk_bytes = staged_chunk(self.n, self.n_pad, self.world, self.mem_size, self.batch,
                                                      self.seg, experiment)
            self._chunks = [torch.empty(self.chunk_bytes, dtype=torch.uint8, device=self.device) for _ in range(2)]
            # the pack's per-tile record counts: written by the counter-based draw of each segment
            # (a buffer per drawn segment, as idx), or by the pack's own count pass (MT draws)
            nt = -(-self.seg * self.batch // 256)
            self._tiles = [torch.empty(nt, dtype=torch.int32, device=self.device)
                           for _ in range(4 if sampler == "philox" else 1)]
            self._gathered = ([torch.empty(self.world * self.chunk_bytes, dtype=torch.uint8, device=self.device)
                               for _ in range(2)] if self.world > 1 else self._chunks)
        self.standin = dict(standin) if standin is not None else None
        if self.standin is not None and not self.emulated:
            nb16 = -(-int(self.standin["bytes"]) // 16) * 16
            self.standin["bytes"] = nb16
            self._standin_src = torch.zeros(nb16, dtype=torch.uint8, device=self.device)
            self._standin_dst = torch.empty(nb16, dtype=torch.uint8, device=self.device)
        self._peers_filled = False
        self.drawn = 0   # segments whose learns are drawn

    @property
    def stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    def _draw(self) -> None:
        g = self.drawn
        if self.sampler == "philox":
            # segment g's draws, marking its rows in segments g - 1 and g (segment g - 1's
            # marks are complete after it). The buffer is zero: the launch that read it last
            # (segment g - 3) cleared it, and begin() clears all three
            nb = self.N_BUFFERS
            tiles = self._tiles[g % 4].data_ptr() if self.exchange == "allgather" else None
            _lib.check(self.lib.sacenv_replay_stage_draw_ctr(
                self._pp, self._spp, g, self.batch, self.seg, self.seed & 0xFFFFFFFFFFFFFFFF,
                self._idx[g % 4].data_ptr(), self.marks[(g - 1) % nb].data_ptr() if g > 0 else None,
                self.marks[g % nb].data_ptr(), tiles, self.stream))
        else:
            _lib.check(self.lib.sacenv_replay_stage_draw(
                self._pp, self._rb.arena.data_ptr(), self._spp, g, self.batch, self.seg,
                self._idx[g % 4].data_ptr(), self._scratch.data_ptr(), self._scratch.numel(), self.stream))
        self.drawn += 1

    def _mark(self, g: int) -> None:
        if self.sampler == "philox":  # (the draws marked the rows)
            return
        _lib.check(self.lib.sacenv_replay_stage_mark(
            self._pp, self._spp, g, self._idx[g % 4].data_ptr(), self._idx[(g + 1) % 4].data_ptr(),
            self.batch, self.seg, self.marks[g % self.N_BUFFERS].data_ptr(), self.stream))

    def begin(self, obs: torch.Tensor) -> None:
        """The buffer starts empty here: the obs every env starts from (the s of its first
        stored transition) go into the last row of the buffer standing for segment -1,
        with term 0; segment 0 and 1's learns are drawn and segment 0's rows marked."""
        nb = self.N_BUFFERS
        last = self.stage[(-1) % nb].view(torch.float32).view(self.n_pad, self.seg, 16)[:, self.seg - 1]
        last.zero_()
        last[: self.n, : _lib.OBS_DIM].copy_(obs.to(device=self.device, dtype=torch.float32))
        for m in self.marks:
            m.zero_()
        self.drawn = 0
        self.prepare(0)

    def stage_args(self, g: int) -> dict:
        """The staged-row arguments of segment g's launch (VecBoatEnv.segment_async /
        sacenv_boat_segment): its 64-B row buffer and the marks of the rows to write."""
        return {"stage": self.stage[g % self.N_BUFFERS], "marks": self.marks[g % self.N_BUFFERS]}

    def prepare(self, g: int) -> None:
        """Before segment g's launch (after segment g - 1's, whose pack reads the buffers
        it reuses): draw the learns up to segment g + 1 and complete segment g's marks."""
        while self.drawn < g + 2:
            self._draw()
        self._mark(g)

    def sample_segment(self, g: int):
        """Enqueue segment g's learns' batches (after its launch, on this stream); returns
        [(state, action, reward f64, new_state, terminal int32 0/1, idx)], one per learn,
        views valid until ``sample_segment(g + 2)``. = ``pack_segment(g)``,
        ``collect_segment(g)``, ``unpack_segment(g)`` on one stream."""
        self.pack_segment(g)
        self.collect_segment(g)
        return self.unpack_segment(g)

    @property
    def fused(self) -> bool:
        """A segment's side work is one launch (``side_segment``): the counter-based draws
        and the all-gather pack/unpack (sacenv_replay_stage_side)."""
        return self.sampler == "philox" and self.exchange == "allgather"

    def side_segment(self, g: int, unpack: int | None = None):
        """After segment g's launch, ONE launch (sacenv_replay_stage_side) doing the unpack
        of segment ``unpack``'s collected chunks (its collective complete in stream
        order), the pack of segment g (``pack_segment``) and ``prepare(g + 1)``'s draws
        (segment g + 2): the same bytes as the three separate calls. Then
        ``collect_segment(g)``; segment g's unpack goes into the next call (or
        ``unpack_segment``). Returns segment ``unpack``'s batches (or None)."""
        if not self.fused:
            raise ValueError("side_segment needs sampler='philox' and exchange='allgather'")
        g = int(g)
        while self.drawn < g + 2:   # (begin() drew 0 and 1; each call draws one more)
            self._draw()
        nb = self.N_BUFFERS
        w = _lib.StageSide()
        d = self.drawn
        draw = d == g + 2
        w.draw_g = d if draw else -1
        if draw:
            w.seed = self.seed & 0xFFFFFFFFFFFFFFFF
            w.draw_idx = self._idx[d % 4].data_ptr()
            w.marks_prev = self.marks[(d - 1) % nb].data_ptr() if d > 0 else None
            w.marks_cur = self.marks[d % nb].data_ptr()
            w.draw_tiles = self._tiles[d % 4].data_ptr()
        w.pack_g = g
        w.stage_cur, w.stage_prev = self.stage[g % nb].data_ptr(), self.stage[(g - 1) % nb].data_ptr()
        w.pack_idx, w.pack_tiles = self._idx[g % 4].data_ptr(), self._tiles[g % 4].data_ptr()
        w.cap, w.chunk = self.cap, self._chunks[g % 2].data_ptr()
        if unpack is not None:
            u = int(unpack)
            w.gathered, w.chunk_bytes = self._gathered[u % 2].data_ptr(), self.chunk_bytes
            w.words, w.status_word, w.world = self._words[u % 2][0].data_ptr(), self._status.data_ptr(), self.world
        _lib.check(self.lib.sacenv_replay_stage_side(self._pp, self._spp, self.batch, self.seg, C.byref(w),
                                                     self.stream))
        if draw:
            self.drawn += 1
        return self._batches[u % 2, u % 4] if unpack is not None else None

    def pack_segment(self, g: int) -> None:
        """This rank's share of segment g's batches, from the staged rows of segments g
        and g - 1 (after segment g's launch): the packed chunk of its rows (all-gather), or
        its rows in the batch words with the others' zero (all-reduce)."""
        g = int(g)
        idx = self._idx[g % 4]
        nb = self.N_BUFFERS
        cur, prev = self.stage[g % nb].data_ptr(), self.stage[(g - 1) % nb].data_ptr()
        if self.exchange == "allgather":
            counted = self.sampler == "philox"   # (the draw of segment g counted its tiles)
            _lib.check(self.lib.sacenv_replay_stage_pack(
                self._pp, self._spp, g, cur, prev, idx.data_ptr(), self.batch, self.seg, self.cap,
                self._chunks[g % 2].data_ptr(), self._tiles[g % 4 if counted else 0].data_ptr(), int(counted),
                self.stream))
        else:
            _lib.check(self.lib.sacenv_replay_sample_staged(
                self._pp, self._spp, g, cur, prev, idx.data_ptr(), self.batch, self.seg,
                self._words[g % 2][0].data_ptr(), self.stream))

    def collect_segment(self, g: int) -> None:
        """The collective over the ranks of segment g's packed share (world > 1): the
        all-gather of the chunks or the SUM all-reduce of the words; at world 1 the
        stand-in for it, if one was asked for."""
        import torch.distributed as dist
        g = int(g)
        if self.emulated:
            if not self._peers_filled:
                self._fill_peers(g)
            sd, cb = self.standin, self.chunk_bytes
            out = self._gathered[g % 2][self.rank * cb:(self.rank + 1) * cb]
            _lib.check(self.lib.sacenv_copy_standin(
                self._chunks[g % 2].data_ptr(), out.data_ptr(), cb, int(sd["workgroups"]), float(sd["us"]),
                self.stream))
        elif self.world > 1:
            if self.exchange == "allgather":
                all_gather_bytes(self._gathered[g % 2], self._chunks[g % 2], self.group)
            else:
                dist.all_reduce(self._words[g % 2][0], op=dist.ReduceOp.SUM, group=self.group)
        elif self.standin is not None:
            sd = self.standin
            _lib.check(self.lib.sacenv_copy_standin(
                self._standin_src.data_ptr(), self._standin_dst.data_ptr(), sd["bytes"], int(sd["workgroups"]),
                float(sd["us"]), self.stream))

    def _fill_peers(self, g: int) -> None:
        """(emulated rank) The other ranks' chunks of both gathered buffers: segment g's
        draws packed from this GPU's staged rows as if its envs were rank r's (each
        rank's slots, counts and record layout as that rank would send them; the values
        are this GPU's rows, not the other ranks' transitions: timing only)."""
        nb, cb = self.N_BUFFERS, self.chunk_bytes
        scratch = torch.empty_like(self._tiles[0])
        for r in range(self.world):
            if r == self.rank:
                continue
            sp = _lib.StagedParams.from_buffer_copy(self.sp)
            sp.offset = r * self.n
            for b in range(2):
                dst = self._gathered[b][r * cb:(r + 1) * cb]
                _lib.check(self.lib.sacenv_replay_stage_pack(
                    self._pp, C.byref(sp), int(g), self.stage[g % nb].data_ptr(), self.stage[(g - 1) % nb].data_ptr(),
                    self._idx[g % 4].data_ptr(), self.batch, self.seg, self.cap, dst.data_ptr(), scratch.data_ptr(),
                    0, self.stream))
        self._peers_filled = True

    def unpack_segment(self, g: int):
        """Segment g's batches from the collected chunks (all-gather; the all-reduce's words
        are the batches already): the views ``sample_segment`` returns."""
        g = int(g)
        if self.exchange == "allgather":
            _lib.check(self.lib.sacenv_replay_stage_unpack(
                self.world, self.chunk_bytes, self.cap, self.batch, self.seg, self._gathered[g % 2].data_ptr(),
                self._words[g % 2][0].data_ptr(), self._status.data_ptr(), self.stream))
        return self._batches[g % 2, g % 4]

    @property
    def bytes_per_segment(self) -> int:
        """The collective's payload of one segment: the all-reduced words, or the
        all-gathered chunks (world x chunk)."""
        if self.exchange == "allgather":
            return self.world * self.chunk_bytes
        return int(self._words[0][0].numel()) * 4

    @property
    def bus_bytes_per_segment(self) -> float:
        """Bytes one rank sends per segment in a ring schedule: 2 (W-1)/W x payload for the
        all-reduce, (W-1) chunks for the all-gather."""
        w = self.world
        if self.exchange == "allgather":
            return float((w - 1) * self.chunk_bytes)
        return 2.0 * (w - 1) / w * self.bytes_per_segment

    def check(self) -> None:
        """Synchronise and raise if a draw ran short of generated MT words (the planned
        5 % margin is > 100 standard deviations of the count at the bench's shape) or a
        rank's packed rows overflowed its chunk (8 standard deviations)."""
        if self._rb is not None and int(self._rb.mt_pos.item()) < 0:
            raise _lib.SacenvError("staged draw: too few MT words generated; the sampling stream is invalid")
        if int(self._status[0].item()) != 0:
            raise _lib.SacenvError("staged all-gather: a rank's rows overflowed its chunk; batches are invalid")


def staged_chunk(n: int, n_pad: int, world: int, mem_size: int, batch: int, seg: int,
                 experiment: int = 6) -> tuple[int, int]:
    """(records, bytes) of one rank's all-gather chunk for this shape
    (``sacenv_replay_stage_chunk``): the same on every rank."""
    lib = _lib.load()
    p = _lib.ReplayParams()
    p.mem_size, p.obs_dim, p.act_dim, p.reward_f32, p.terminal_mask = int(mem_size), _lib.OBS_DIM, 1, 1, 2
    sp = _lib.StagedParams()
    sp.period, sp.offset, sp.n, sp.n_pad, sp.seg, sp.experiment = world * n, 0, n, n_pad, seg, experiment
    cap, nbytes = C.c_int64(), C.c_int64()
    _lib.check(lib.sacenv_replay_stage_chunk(C.byref(p), C.byref(sp), int(batch), int(seg), C.byref(cap),
                                             C.byref(nbytes)))
    return int(cap.value), int(nbytes.value)


def all_gather_bytes(out: torch.Tensor, chunk: torch.Tensor, group=None) -> None:
    """out [world x chunk] = every rank's chunk in rank order: all_gather_into_tensor over
    RCCL; gloo (rehearsals) through the list form."""
    import torch.distributed as dist
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, chunk, group=group)
    else:
        dist.all_gather(list(out.chunk(dist.get_world_size(group))), chunk, group=group)


class ReplayBuffer:
    """Drop-in for agent.buffer.ReplayBuffer (buffer.py:3-35), GPU-backed, numpy I/O,
    sampling from numpy's global RNG stream like ``np.random.choice`` (buffer.py:27)."""

    def __init__(self, max_size, input_shape, n_actions, *, device=None):
        self._rb = DeviceReplayBuffer(max_size, input_shape, n_actions, device=device,
                                      reward_f32=False, terminal_mask=TERMINAL_GOAL)
        self.mem_size = self._rb.mem_size

    @property
    def mem_cntr(self) -> int:
        return self._rb.mem_cntr

    def store_transition(self, state, action, reward, state_, done):
        rb = self._rb
        one = lambda x, dt: np.asarray(x, dtype=dt).reshape(1, -1)  # noqa: E731
        rb.store_batch(torch.from_numpy(one(state, np.float32)), torch.from_numpy(one(action, np.float32)),
                       torch.tensor([float(reward)], dtype=torch.float64),
                       torch.from_numpy(one(state_, np.float32)),
                       torch.tensor([1 if done else 0], dtype=torch.uint8))

    def sample_buffer(self, batch_size):
        rb = self._rb
        st = np.random.get_state(legacy=True)
        rb.mt_key.copy_(torch.from_numpy(np.asarray(st[1], dtype=np.uint32).view(np.int32)))
        rb.mt_pos.fill_(int(st[2]))
        states, actions, rewards, states_, dones, _ = rb.sample(batch_size)
        torch.cuda.synchronize(rb.device)
        key = rb.mt_key.cpu().numpy().view(np.uint32).copy()
        np.random.set_state((st[0], key, int(rb.mt_pos.item()), st[3], st[4]))
        # the reference's memory arrays are float64 (np.zeros default, buffer.py:7-10)
        return (states.cpu().numpy().astype(np.float64), actions.cpu().numpy().astype(np.float64),
                rewards.cpu().numpy(), states_.cpu().numpy().astype(np.float64), dones.cpu().numpy())


__all__ = ["DeviceReplayBuffer", "ReplayBuffer", "ShardedReplayBuffer", "StagedReplay", "TERMINAL_GOAL",
           "staged_chunk", "all_gather_bytes"]
