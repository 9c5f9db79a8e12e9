#!/bin/bash
# Full GPU check: parity tests (log kept), then the bench configs of BASELINE.json.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1200 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
B="timeout -k 10 300 python bench.py"
$B --no-cpu-baseline > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.log || exit 1
$B --mixed --cpu-seconds 10 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.log || exit 1
$B --experiment 1 --envs 4096 --cpu-seconds 10 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.log || exit 1
for f in c3 c5 c2; do python -c "import json;d=json.load(open('gpurun_out/bench_$f.json'));print('$f', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step']*1e3,2), 'us/step', 'frac', round(d['roofline']['frac'],3), 'cpu', d['cpu_baseline'] and round(d['cpu_baseline']['value']))"; done
