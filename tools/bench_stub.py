"""bench.py --stub: its control flow on the CPU with no kernels (tests, rehearsals).

A stub workload stands in for the HIP engine: ``StubEnv`` has the record and
terminal-obs regions the pooling reads and counts steps and refills;
``StubSampler`` stands in for ``sacenv.replay.StagedReplay`` (the rows it is
handed and one SUM all-reduce of a segment's packed batches over the ranks).
Every line bench.py prints from this mode says ``"data": "stub ..."`` -- it
measures the harness, not the engine.
"""
from __future__ import annotations

import torch

N_ENVS, N_PAD = 70, 128


class StubEnv:
    """Stands in for VecBoatEnv: the record / terminal-obs regions the pool reads."""

    def __init__(self, rank):
        self.num_envs, self.n_pad = N_ENVS, N_PAD
        self.record = torch.zeros(50 * N_PAD, dtype=torch.uint8)
        self.final_obs_bytes = torch.zeros(44 * N_PAD, dtype=torch.uint8)
        self.obs = torch.zeros(N_ENVS, 11)
        self.rank, self.steps, self.refills, self.refill_at = rank, 0, 0, []

    def step_async(self, actions):
        assert actions.dtype == torch.float32 and actions.numel() == N_ENVS
        self.steps += 1
        self.record.fill_((self.steps + 31 * self.rank) % 251)
        self.final_obs_bytes.fill_((self.steps * 7 + self.rank) % 253)

    def refill(self):
        self.refills += 1
        self.refill_at.append(self.steps)


class StubSampler:
    """Stands in for StagedReplay: three row buffers, one collective per segment (the
    all-gather of a fixed chunk per rank, or the SUM all-reduce of the batch words)."""

    def __init__(self, row_bytes, seg, batch, world, n_buffers=3, exchange="allgather"):
        self.row_bytes, self.seg, self.batch, self.world = row_bytes, seg, batch, world
        self.exchange = exchange
        self.buffers = [torch.zeros(seg * row_bytes, dtype=torch.uint8) for _ in range(n_buffers)]
        self.words = torch.zeros(seg * batch * 26, dtype=torch.int32)
        self.chunk = torch.zeros(-(-seg * batch // world) * 25 + 4, dtype=torch.int32)
        self.gathered = torch.zeros(world * self.chunk.numel(), dtype=torch.int32)
        self.sampled = []

    def stage_args(self, g):
        return {"rows": self.buffers[g % len(self.buffers)]}

    def begin(self, obs):
        self.sampled.clear()

    def prepare(self, g):
        pass

    def sample_segment(self, g):
        import torch.distributed as dist
        if self.exchange == "allgather":
            self.chunk.fill_(g)
            if self.world > 1:
                dist.all_gather(list(self.gathered.chunk(self.world)), self.chunk)
        else:
            self.words.fill_(g)
            if self.world > 1:
                dist.all_reduce(self.words)
        self.sampled.append(g)
        return []

    @property
    def bytes_per_segment(self):
        return (self.gathered.numel() if self.exchange == "allgather" else self.words.numel()) * 4

    @property
    def bus_bytes_per_segment(self):
        w = self.world
        if self.exchange == "allgather":
            return float((w - 1) * self.chunk.numel() * 4)
        return 2.0 * (w - 1) / w * self.bytes_per_segment

    def check(self):
        pass


def workload(bench, rank):
    """(StubEnv, bench.Workload) of one rank."""
    from sacenv.dist import TransitionLayout
    env = StubEnv(rank)
    actions = torch.rand((bench.ACTION_STEPS, N_ENVS), generator=torch.Generator().manual_seed(rank))
    lay = TransitionLayout(N_ENVS, N_PAD)

    def pooled_step(k, row):
        assert row.numel() == lay.nbytes
        env.step_async(actions[k % bench.ACTION_STEPS])
        row.fill_((env.steps * 3 + rank) % 255)

    return env, bench.Workload([env], env.step_async, env.refill, actions, pooled_step, lay.nbytes,
                               N_ENVS, bench.BYTES_PER_ENV_STEP * N_ENVS)
