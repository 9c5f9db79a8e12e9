#!/bin/bash
# GPU session script: parity tests, phase stamps, bench variants.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 180 python tools/stamps.py --rebuild > gpurun_out/stamps_tm0.txt 2>&1 || exit 1
cat gpurun_out/stamps_tm0.txt
B="timeout -k 10 120 python bench.py --steps 1000 --warmup 200 --no-cpu-baseline"
$B > gpurun_out/sw_default.json 2>/dev/null || exit 1
cat gpurun_out/sw_default.json
$B --helpers 128 > gpurun_out/sw_h128.json 2>/dev/null || exit 1
cat gpurun_out/sw_h128.json
echo sweep done
