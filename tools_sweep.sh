#!/bin/bash
# bench sweep (diagnostics): variants that isolate the step from the resets
set -o pipefail
mkdir -p gpurun_out
B="timeout -k 10 120 python bench.py --steps 1000 --warmup 200 --no-cpu-baseline"
$B > gpurun_out/sw_default.json 2>/dev/null || exit 1
$B --test-mode 1 --episode-steps 0 > gpurun_out/sw_tm1_exp6.json 2>/dev/null || exit 1
$B --test-mode 1 --episode-steps 0 --experiment 1 > gpurun_out/sw_tm1_exp1.json 2>/dev/null || exit 1
$B --test-mode 1 --episode-steps 0 --envs 262144 > gpurun_out/sw_tm1_exp6_262k.json 2>/dev/null || exit 1
$B --envs 262144 > gpurun_out/sw_default_262k.json 2>/dev/null || exit 1
$B --episode-steps 0 > gpurun_out/sw_notrunc.json 2>/dev/null || exit 1
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r01 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1000 --warmup 200 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_bench.json 2>$GRAFT_REPO_ROOT/gpurun_out/prof_err.log || exit 1
echo sweep done
