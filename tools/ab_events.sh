set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2 3; do for e in 1 1000 4; do
timeout -k 10 120 python bench.py --no-cpu-baseline --event-every $e > gpurun_out/ev_$e.json 2> gpurun_out/ev_$e.log || { tail -5 gpurun_out/ev_$e.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/ev_$e.json'));r=d['roofline'];print('r$r ev$e', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step']*1e3,3),'us/step kernel', round(r['kernel_avg_us'],3), r['timing'][:40])"
done; done
