set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.log || exit 1
python -c "import json;d=json.load(open('gpurun_out/bench_default.json'));print(round(d['value']/1e9,3), 'G/s', round(d['ms_per_step']*1e3,3), 'us/step', 'k_step', round(d['roofline']['kernel_avg_us'],3), 'frac', round(d['roofline']['frac'],3))"
