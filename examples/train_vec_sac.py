"""Device-resident SAC training loop over N boat envs.

main.py:70-114 for N envs at once, every tensor on the GPU:

* ``VecSAC.choose_action`` acts on all N observations ([N, 11] -> [N, 1]);
* ``VecBoatEnv`` steps all envs in one kernel (auto-reset in-kernel);
* ``DeviceReplayBuffer.store_env_step`` appends the N transitions in one launch,
  terminal as main.py:83-88 stores it (the env's persistent last termination);
* ``VecSAC.learn`` is ContinuousAgent.learn (continuous_agent.py:96-154) on a
  1 024-row batch sampled on the device (pinned to the reference by
  tests/test_agent_cpu.py).

``--agent native`` (default) runs choose_action and learn on the fp32 MFMA
kernels of sacenv_sac.hip (``NativeSAC``, checked against VecSAC by
tests/test_sac_native_gpu.py); ``--agent torch`` on VecSAC.

    python examples/train_vec_sac.py --envs 65536 --iters 200 [--agent torch]

Prints one JSON line: env-steps/s of the whole loop (act + step + store +
sample + update), and the env step's share of it.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sac-agent_amd"))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--learn-every", type=int, default=1)
    ap.add_argument("--agent", choices=("native", "torch"), default="native")
    args = ap.parse_args(argv)
    from sacenv import VecBoatEnv
    from sacenv.agent import VecSAC
    from sacenv.sac_native import NativeSAC
    dev = torch.device("cuda")
    env = VecBoatEnv({"base_settings": {"experiment": 6, "test_mode": 0}}, args.envs, seed=0,
                     device=dev, max_episode_steps=500)
    agent = (NativeSAC if args.agent == "native" else VecSAC)(dev, init_seed=0)
    obs = env.reset().clone()
    losses = None

    def iteration(i):
        nonlocal obs, losses
        a = agent.choose_action(obs)
        env.step(a.view(-1))
        agent.memory.store_env_step(obs, a, env)
        obs = env.obs.clone()
        if i % args.learn_every == 0:
            out = agent.learn()
            losses = out if out is not None else losses

    for i in range(5):
        iteration(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.iters):
        iteration(i)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    # the env step alone, same shapes
    a = torch.zeros(args.envs, device=dev)
    t1 = time.perf_counter()
    for _ in range(args.iters):
        env.step_async(a)
    torch.cuda.synchronize()
    el_env = time.perf_counter() - t1
    out = {"pipeline": "act + VecBoatEnv.step + replay store + sample(1024) + SAC update",
           "agent": args.agent, "envs": args.envs, "iters": args.iters,
           "env_steps_per_s": args.envs * args.iters / el, "ms_per_iter": el / args.iters * 1e3,
           "env_step_ms": el_env / args.iters * 1e3,
           "losses": None if losses is None else [float(x) for x in losses]}
    print(json.dumps(out))
    return out


if __name__ == "__main__":
    main()
