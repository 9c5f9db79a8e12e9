set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
VARIANTS="base" bash tools/ab.sh || exit 1
for a in "--no-autoreset" "--test-mode 1 --episode-steps 0"; do
  timeout -k 10 120 python bench.py --steps 2000 --warmup 300 --no-cpu-baseline $a > gpurun_out/d.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/d.json'));r=d['roofline'];print('$a', round(r['step_us_incl_refill'],3), 'kstep', round(r['kernel_avg_us'],3))"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 1024 > $GRAFT_REPO_ROOT/gpurun_out/bp.json 2>$GRAFT_REPO_ROOT/gpurun_out/bp.log || exit 1
cd $GRAFT_REPO_ROOT && python -c "
import csv,glob
for r in csv.DictReader(open(glob.glob('gpurun_out/prof/**/*kernel_stats.csv',recursive=True)[0])):
    print(r['Name'][:50], r['Calls'], r['AverageNs'], r['MinNs'], r['MaxNs'])
"
