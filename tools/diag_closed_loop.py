"""Diagnostic (round 4): the closed loop's hand-off step by step at a small size --
flags, status and action rows after each stage."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sac-agent_amd"))
import torch  # noqa: E402

from sacenv import VecBoatEnv  # noqa: E402
from sacenv.closed_loop import ClosedLoop  # noqa: E402
from sacenv.sac_native import NativeSAC  # noqa: E402

dev = torch.device("cuda", 0)
N, K = int(os.environ.get('DIAG_N', 256)), int(os.environ.get('DIAG_K', 4))
env = VecBoatEnv({"base_settings": {"experiment": 6, "test_mode": 0}}, N, seed=5, device=dev,
                 max_episode_steps=60, n_helpers=64, auto_refill=False)
env.reset()
agent = NativeSAC(dev, init_seed=3, with_memory=False)
loop = ClosedLoop(env, agent, segment=K)
print("plan", loop.plan)
eps = torch.randn((K, N), device=dev)
# the policy alone, flags pre-published: rows 0..K-1
st = torch.zeros(N // 64, dtype=torch.int32, device=dev) + (1 << 20)
ar = torch.zeros(N // 64, dtype=torch.int32, device=dev)
out = torch.zeros((K, N), device=dev)
for k in range(K):
    agent.choose_action_handoff(env.obs, eps[k], out[k], obs_ready=st, obs_want=k, act_ready=ar, act_value=k + 1,
                                status=env.status[1:2])
torch.cuda.synchronize()
print("policy alone: act_ready", sorted(set(ar.tolist())), "rows nonzero", [(out[k] != 0).sum().item() for k in range(min(K, 8))],
      "status", env.status[1].item())
ref = torch.stack([agent.choose_action(env.obs, eps=eps[k]).reshape(-1) for k in range(K)])
torch.cuda.synchronize()
print("policy alone == choose_action:", torch.equal(out, ref))
import time
t0 = time.perf_counter()
loop.run(eps)
torch.cuda.synchronize()
print("loop time", time.perf_counter() - t0)
print("loop: step_done", loop.step_done.tolist(), "act_ready", loop.act_ready.tolist(), "status",
      env.status[1].item(), "rows nonzero", [(loop.actions[k] != 0).sum().item() for k in range(min(K, 8))])
print("step_done set", sorted(set(loop.step_done.tolist()))[:8], "act_ready set", sorted(set(loop.act_ready.tolist()))[:8])
