set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 bash tools/pmc.sh > gpurun_out/pmc_run.log 2>&1 || { tail -30 gpurun_out/pmc_run.log; exit 1; }
tail -25 gpurun_out/pmc_run.log | head -24
B="timeout -k 10 300 python bench.py"
$B --mixed --cpu-seconds 10 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.log || exit 1
$B --experiment 1 --envs 4096 --cpu-seconds 10 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.log || exit 1
$B --rollout 128 --steps 2048 --warmup 256 --no-cpu-baseline > gpurun_out/roll_128.json 2> gpurun_out/roll_128.log || exit 1
for f in c5 c2; do python -c "import json;d=json.load(open('gpurun_out/bench_$f.json'));print('$f', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step']*1e3,2), 'us/step', 'frac', round(d['roofline']['frac'],3), 'cpu', d['cpu_baseline'] and round(d['cpu_baseline']['value']))"; done
