"""Env-instance data parallelism across the GPUs of a node.

Envs are independent (no cross-env term in BoatEnv.step), so each rank owns
a contiguous block of global env ids [rank*N, (rank+1)*N) and seeds every env
by its GLOBAL id: results do not depend on the world size. The only
collective is one all-gather per step of the packed per-env record that the
step kernel already writes contiguously (VecBoatEnv.record):

    [ obs f32 N x 11 | reward f32 N | done u8 N | term u8 N ]  = 50 B/env

so the gather needs no packing kernel. Over RCCL (backend "nccl") this is
``all_gather_into_tensor``; gloo (CPU tests) falls back to list all_gather.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

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
