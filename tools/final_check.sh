#!/bin/bash
# Round-end evidence on one GPU box, each GPU step under its own time limit,
# the first failure ends the script:
#   parity tests (log kept), smoke(), the driver's bench command, the default
#   bench line with cpu_baseline, the config lines (C2 per step and as K-step
#   rollouts, C5 mixed, the K=128 rollout), phase stamps, then tools/pmc.sh
#   (kernel trace + calibrated PMC passes).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
tail -1 gpurun_out/smoke.log
B="timeout -k 10 300 python bench.py"
$B --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.json 2> gpurun_out/bench_driver.log || exit 1
$B > gpurun_out/bench_default.json 2> gpurun_out/bench_default.log || exit 1
$B --experiment 1 --envs 4096 --cpu-seconds 6 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.log || exit 1
$B --experiment 1 --envs 4096 --rollout 128 > gpurun_out/bench_c2_rollout.json 2> gpurun_out/bench_c2_rollout.log || exit 1
$B --mixed --cpu-seconds 6 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.log || exit 1
$B --rollout 128 > gpurun_out/bench_rollout_k128.json 2> gpurun_out/bench_rollout_k128.log || exit 1
$B --envs 131072 --no-cpu-baseline > gpurun_out/bench_131k.json 2> gpurun_out/bench_131k.log || exit 1
python - <<'PY'
import json
for f in ("driver", "default", "c2", "c2_rollout", "c5", "rollout_k128", "131k"):
    d = json.load(open(f"gpurun_out/bench_{f}.json"))
    r, c = d["roofline"], d.get("cpu_baseline")
    k = r.get("kernel_avg_us", r.get("kernel_avg_us_per_step"))
    print(f"{f:13s} {d['value']/1e9:7.3f} G/s {d['ms_per_step']*1e3:6.2f} us/step kernel {k:5.2f} us "
          f"frac {r['frac']:.3f} cpu {c and round(c['value'])}")
PY
timeout -k 10 300 python tools/stamps.py --rebuild > gpurun_out/stamps_full.txt 2>&1 || exit 1
bash tools/pmc.sh > gpurun_out/pmc.log 2>&1 || { tail -20 gpurun_out/pmc.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/pmc_k_step.json'));print('pmc', d['trace_avg_ns'], d['hbm_bytes_per_launch'])"
echo final_check done
