set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
VARIANTS="base" bash tools/ab.sh || exit 1
timeout -k 10 200 python bench.py --rollout 128 --steps 2048 --warmup 256 --no-cpu-baseline > gpurun_out/roll_128.json 2> gpurun_out/roll_128.log || exit 1
python -c "import json;d=json.load(open('gpurun_out/roll_128.json'));r=d['roofline'];print('rollout K=128', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step']*1e3,3), 'us/step kernel', round(r['kernel_avg_us_per_step'],3))"
