#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for v in base prio; do
    for ov in 0 1; do
      if [ "$v" = base ]; then unset SACENV_LIB; else export SACENV_LIB=$PWD/sac-agent_amd/build/libsacenv_$v.so; fi
      timeout -k 10 200 python bench.py --no-cpu-baseline --refill-overlap $ov > gpurun_out/abp.json 2> gpurun_out/abp.log || { tail -5 gpurun_out/abp.log; exit 1; }
      unset SACENV_LIB
      python -c "import json;d=json.load(open('gpurun_out/abp.json'));r=d['roofline'];print('r$r $v overlap=$ov', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step']*1e3,3), 'us/step; kernel', round(r['kernel_avg_us'],3), 'incl refill', round(r['step_us_incl_refill'],3))"
    done
  done
done
