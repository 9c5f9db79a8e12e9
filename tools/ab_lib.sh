#!/bin/bash
# A/B of library variants (tools/variant.py) on one box: the bench line per variant,
# alternating rounds. VARIANTS="base v1 v2"; base = the in-tree library.
set -o pipefail
mkdir -p gpurun_out
ARGS=${BENCH_ARGS:-"--no-cpu-baseline"}
for round in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARIANTS:-base}; do
    if [ "$v" = base ]; then unset SACENV_LIB; else export SACENV_LIB=$PWD/sac-agent_amd/build/libsacenv_$v.so; fi
    timeout -k 10 200 python bench.py $ARGS > gpurun_out/abl_$v.json 2> gpurun_out/abl_$v.log || { tail -5 gpurun_out/abl_$v.log; exit 1; }
    unset SACENV_LIB
    python -c "import json;d=json.load(open('gpurun_out/abl_$v.json'));r=d['roofline'];print('r$round $v', round(d['value']/1e9,3), 'G/s', round(r['kernel_avg_us'],3), 'us/step kernel', round(r['step_us_incl_refill'],3), 'replay', round((d.get('replay_path') or {}).get('value',0)/1e9,3), 'every', round((d.get('every_output') or {}).get('value',0)/1e9,3))"
  done
done
