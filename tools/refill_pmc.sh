#!/bin/bash
# Refill characterisation on one GPU box: two SQ counter passes over the eager bench
# (k_refill / k_refill_fit instruction mix and wait cycles), then the number of envs
# each 128-step segment refills (status word 2 after sacenv_boat_refill).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p "$OUT"
BENCH="python3 bench.py --steps 256 --warmup 128 --no-cpu-baseline --no-graph"
i=0
while read -r c; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $c -d "$OUT/rf_pmc$i" -o run --output-format csv -- $BENCH > /dev/null 2> "$OUT/rf_pmc$i.log" || exit 1
done <<'LIST'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU
SQ_WAIT_ANY SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_INSTS_SMEM
LIST
timeout -k 10 120 python3 - <<'PY'
import sys, torch
sys.path.insert(0, "sac-agent_amd")
from sacenv import VecBoatEnv
N = 65536
env = VecBoatEnv({"base_settings": {"experiment": 6, "test_mode": 0}}, N, seed=0, device="cuda",
                 autoreset=True, max_episode_steps=500, auto_refill=False)
env.reset()
g = torch.Generator(device="cuda"); g.manual_seed(1)
for seg in range(12):
    for k in range(128):
        env.step_async(torch.rand(N, device="cuda", generator=g) * 2 - 1) if hasattr(env, "step_async") else env.step(torch.rand(N, device="cuda", generator=g) * 2 - 1)
    env.refill(); torch.cuda.synchronize()
    print("segment", seg, "refilled envs", int(env.status[2].item()))
PY
echo ok
