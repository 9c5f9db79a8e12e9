set -o pipefail
mkdir -p gpurun_out
B="timeout -k 10 120 python bench.py --steps 2000 --warmup 300 --no-cpu-baseline"
for a in "" "--no-autoreset" "--test-mode 1 --episode-steps 0" "" "--no-autoreset"; do
  $B $a > gpurun_out/d.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/d.json'));print('$a', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step']*1e3,2), 'us/step kernel', round(d['roofline']['kernel_us_median'],2))"
done
