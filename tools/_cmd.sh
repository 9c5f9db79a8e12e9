set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/b.json 2> gpurun_out/b.log || exit 1
python -c "import json;d=json.load(open('gpurun_out/b.json'));r=d['roofline'];print('bench', round(d['value']/1e9,3), 'G/s step', round(r['step_us_incl_refill'],3), 'kstep', round(r['kernel_avg_us'],3), 'frac', round(r['frac'],4))"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 1024 > $GRAFT_REPO_ROOT/gpurun_out/bp.json 2>$GRAFT_REPO_ROOT/gpurun_out/bp.log || exit 1
cd $GRAFT_REPO_ROOT && find gpurun_out/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} python -c "
import csv,sys
for r in csv.DictReader(open('{}')):
    print(r['Name'][:60], r['Calls'], r['AverageNs'], r['MinNs'], r['MaxNs'])
"
