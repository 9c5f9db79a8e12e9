"""ShardedReplayBuffer on the device (sacenv_replay_store_shard / _sample_shard).

Two ranks (gloo, both on the one GPU of the box; the driver's 8-GPU node runs
RCCL) each step their shard of envs (global-id seeds) and store only their own
transitions; rank 0 also runs the pooled reference -- one VecBoatEnv over all
global envs feeding one DeviceReplayBuffer, i.e. the buffer every rank would
hold after all-gathering every transition (main.py:81-88, agent/buffer.py:3-35).
The sharded batches (one integer SUM all-reduce of the owned rows) must equal the
pooled buffer's batches bit for bit, with the ring wrapping (mem_size not a
multiple of the rows per step) and the reference's persistent terminal rule.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "sac-agent_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from sacenv import VecBoatEnv
        from sacenv.replay import DeviceReplayBuffer, ShardedReplayBuffer
        dev = torch.device("cuda", 0)
        N, M, B, steps = 1000 if world == 2 else 500, 4999, 511, 12   # B odd: f64 words stay aligned
        cfg = {"base_settings": {"experiment": 6, "test_mode": 0}, "boat_env": {"track_width": 30}}
        kw = dict(seed=3, device=dev, max_episode_steps=7)
        env = VecBoatEnv(cfg, N, env_id_offset=rank * N, **kw)
        env.reset()
        rb = ShardedReplayBuffer(M, (11,), 1, rank=rank, world=world, envs_per_rank=N, device=dev, seed=5)
        ref = ref_rb = None
        if rank == 0:
            ref = VecBoatEnv(cfg, world * N, **kw)
            ref.reset()
            ref_rb = DeviceReplayBuffer(M, (11,), 1, device=dev, seed=5)
        g = torch.Generator(device=dev)
        g.manual_seed(9)
        checked = 0
        for t in range(steps):
            acts = torch.rand((world * N,), generator=g, device=dev) * 2 - 1
            a = acts[rank * N:(rank + 1) * N].contiguous()
            prev = env.obs.clone()
            env.step(a)
            rb.store_env_step(prev, a, env)
            if ref is not None:
                prev_r = ref.obs.clone()
                ref.step(acts)
                ref_rb.store_env_step(prev_r, acts, ref)
            if t % 3 == 2:
                # one batch, or (every 6th step) three learns' batches in ONE all-reduce
                n_b = 3 if t % 6 == 5 else 1
                gots = rb.sample_many(B, n_b) if n_b > 1 else [rb.sample(B)]
                if ref_rb is not None:
                    for got in gots:
                        want = ref_rb.sample(B)
                        torch.cuda.synchronize()
                        assert torch.equal(got[5], want[5]), "indices"
                        for i, (x, y) in enumerate(zip(got[:5], want[:5])):
                            assert torch.equal(x.reshape(-1), y.reshape(-1).to(x.dtype)), (t, i)
                        checked += 1
        torch.cuda.synchronize()
        q.put((rank, checked))
    except Exception as exc:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_replay_equals_pooled_buffer_gpu(world, gpu, built_lib):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert res[0] == 8 and all(res[r] == 0 for r in range(1, world)), res
