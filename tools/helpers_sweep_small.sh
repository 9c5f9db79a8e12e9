set -o pipefail
mkdir -p gpurun_out
for h in 256 64 32 16; do
  timeout -k 10 120 python bench.py --steps 2000 --warmup 300 --no-cpu-baseline --experiment 1 --envs 4096 --helpers $h > gpurun_out/h.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/h.json'));print('c2 h$h', round(d['value']/1e9,3), 'G/s', round(d['roofline']['kernel_avg_us'],2))"
done
for h in 256 64; do
  timeout -k 10 120 python bench.py --steps 2000 --warmup 300 --no-cpu-baseline --envs 4096 --helpers $h > gpurun_out/h.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/h.json'));print('exp6-4096 h$h', round(d['value']/1e9,3), 'G/s', round(d['roofline']['kernel_avg_us'],2))"
done
