#!/bin/bash
# bench line per refill-helper count (--helpers), alternating rounds
set -o pipefail
mkdir -p gpurun_out
for round in 1 2; do
  for h in ${HELPERS:-8192 12288 16384}; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --helpers $h > gpurun_out/hs_$h.json 2> gpurun_out/hs_$h.log || { tail -5 gpurun_out/hs_$h.log; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/hs_$h.json'));r=d['roofline'];print('r$round helpers $h', round(d['value']/1e9,3), 'G/s', round(r['kernel_avg_us'],3), round(r['step_us_incl_refill'],3))"
  done
done
