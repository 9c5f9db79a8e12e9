#!/bin/bash
# Round-end evidence on one GPU box, each GPU step under its own time limit,
# the first failure ends the script:
#   parity tests (log kept), smoke(), the driver's bench command, the default
#   bench line (persistent segments) with cpu_baseline, the per-step-launch line,
#   the config lines (C2, C5 mixed, 131 072 envs, the K=128 rollout), the N=2
#   rehearsals over gloo on the one GPU (the sharded exchange and the all-gather),
#   the training loop (--train),
#   then tools/pmc.sh (kernel trace + calibrated PMC
#   passes of the persistent segment kernel).
# PART=1: tests, smoke and the bench lines; PART=2: the rest (two gpurun calls).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${PART:-all}
if [ "$P" != 2 ] && [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
  tail -1 gpurun_out/smoke.log
fi
B="timeout -k 10 300 python bench.py"
if [ "$P" != 2 ]; then
$B --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.json 2> gpurun_out/bench_driver.log || exit 1
$B > gpurun_out/bench_default.json 2> gpurun_out/bench_default.log || exit 1
$B --launch step --no-cpu-baseline > gpurun_out/bench_step.json 2> gpurun_out/bench_step.log || exit 1
$B --experiment 1 --envs 4096 --cpu-seconds 6 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.log || exit 1
$B --mixed --cpu-seconds 6 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.log || exit 1
$B --rollout 128 > gpurun_out/bench_rollout_k128.json 2> gpurun_out/bench_rollout_k128.log || exit 1
$B --envs 131072 --no-cpu-baseline > gpurun_out/bench_131k.json 2> gpurun_out/bench_131k.log || exit 1
$B --closed-loop --no-cpu-baseline > gpurun_out/bench_closed.json 2> gpurun_out/bench_closed.log || exit 1
python - <<'PY'
import json
for f in ("driver", "default", "step", "c2", "c5", "rollout_k128", "131k", "closed"):
    d = json.load(open(f"gpurun_out/bench_{f}.json"))
    r, c = d.get("roofline") or {}, d.get("cpu_baseline")
    k = r.get("kernel_avg_us", r.get("kernel_avg_us_per_step")) or 0.0
    print(f"{f:13s} {d['value']/1e9:7.3f} G/s {d['ms_per_step']*1e3:6.2f} us/step kernel {k:5.2f} us "
          f"frac {r.get('frac', 0):.3f} cpu {c and round(c['value'])}")
d = json.load(open("gpurun_out/bench_default.json"))
rp, sd, ev = d["replay_path"], d["replay_path_collective_standin"], d["every_output"]
rk = d["replay_path_rank_of_world"]
print(f"default: replay_path {rp['value']/1e9:.3f} ({rp['value']/d['value']:.3f}), standin {sd['value']/1e9:.3f} "
      f"({sd['value']/d['value']:.3f}), rank_of_{rk['world']} {rk['value']/1e9:.3f} ({rk['value']/d['value']:.3f}), "
      f"every_output {ev['value']/1e9:.3f} ({ev['value']/d['value']:.3f}), "
      f"timed {d['steps'] * d['ms_per_step'] * 1e-3:.3f} s")
PY
fi
[ "$P" = 1 ] && { echo final_check part 1 done; exit 0; }
# N=2 rehearsals over gloo on the one GPU: the default sharded exchange (bench starting its
# own ranks, no launcher), and the all-gather under torch.distributed.run
SACENV_BENCH_BACKEND=gloo SACENV_BENCH_ONE_DEVICE=1 timeout -k 10 400 python bench.py --gpus 2 --envs 65536 \
  --steps 256 --warmup 128 > gpurun_out/rehearse_sharded.json 2> gpurun_out/rehearse_sharded.log \
  || { tail -20 gpurun_out/rehearse_sharded.log; exit 1; }
SACENV_BENCH_BACKEND=gloo SACENV_BENCH_ONE_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run \
  --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 \
  --envs 65536 --pooling gather --steps 256 --warmup 128 > gpurun_out/rehearse_gather.json \
  2> gpurun_out/rehearse_gather.log || { tail -20 gpurun_out/rehearse_gather.log; exit 1; }
python - <<'PY'
import json
for f in ("sharded", "gather"):
    d = json.loads(open(f"gpurun_out/rehearse_{f}.json").read().strip().splitlines()[-1])
    p = d["pooling"]
    print(f"rehearse {f}: {d['value']/1e9:.3f} G/s {d['dist']['backend']} no_exchange "
          f"{p['no_exchange']['value']/1e9:.3f}" + (f" all_gather {p['all_gather']['value']/1e9:.3f}"
                                                  if p.get('all_gather') else ""))
PY
$B --train > gpurun_out/bench_train.json 2> gpurun_out/bench_train.log || exit 1
python -c "import json;d=json.load(open('gpurun_out/bench_train.json'));print('train', round(d['value']/1e6,1), 'M/s', d['parts'])"
bash tools/ktrace.sh > gpurun_out/kt_final.txt 2>&1 || { tail -20 gpurun_out/kt_final.txt; exit 1; }
cat gpurun_out/kt_final.txt
if [ -n "$RUN_PMC" ]; then
  bash tools/pmc.sh > gpurun_out/pmc.log 2>&1 || { tail -20 gpurun_out/pmc.log; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/pmc_segment.json'));print('pmc', d['trace_avg_ns_per_step'], d['hbm_bytes_per_step'])"
fi
echo final_check done
