#!/bin/bash
# GPU session script: parity tests, phase stamps, bench variants.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
[ -n "$SKIP_TESTS" ] || timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
B="timeout -k 10 120 python bench.py --steps 2000 --warmup 300 --no-cpu-baseline"
for v in ${VARIANTS:-base prev}; do
  if [ "$v" != "base" ]; then export SACENV_LIB=$PWD/sac-agent_amd/build/libsacenv_$v.so; else unset SACENV_LIB; fi
  $B > gpurun_out/sw_$v.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/sw_$v.json'));print('$v', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step']*1e3,2), 'us/step kernel', round(d['roofline']['kernel_avg_us'],2))"
done
echo sweep done
