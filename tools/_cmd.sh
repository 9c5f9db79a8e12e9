set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
VARIANTS="base" bash tools/ab.sh || exit 1
timeout -k 10 300 python bench.py --experiment 1 --envs 4096 --no-cpu-baseline > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.log || exit 1
python -c "import json;d=json.load(open('gpurun_out/bench_c2.json'));print('c2', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step']*1e3,2), 'us/step')"
