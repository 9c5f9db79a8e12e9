#!/bin/bash
# GPU check on one box: parity tests (log kept), the driver's bench command and the
# default bench line. Every GPU step has its own time limit; the first failure ends it.
#   TESTS="tests/test_x.py" to run a subset; SKIP_BENCH=1 to stop after the tests.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|error" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
[ -n "$SKIP_BENCH" ] && exit 0
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.json \
  2> gpurun_out/bench_driver.log || { tail -20 gpurun_out/bench_driver.log; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.log \
  || { tail -20 gpurun_out/bench_default.log; exit 1; }
python - <<'PY'
import json
for f in ("driver", "default"):
    d = json.load(open(f"gpurun_out/bench_{f}.json"))
    r, c = d["roofline"], d["cpu_baseline"]
    print(f, f"{d['value']/1e9:.3f} G/s", f"{d['ms_per_step']*1e3:.2f} us/step", f"kernel {r.get('kernel_avg_us')} us",
          f"frac {r['frac']:.3f}", "cpu", c and round(c["value"]), c and c["cores"], c and round(c["one_core"]))
PY
