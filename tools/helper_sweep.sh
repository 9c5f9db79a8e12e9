#!/bin/bash
# k_refill helper count sweep on the default bench line (alternating rounds)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do for h in ${HELPERS:-4096 6144 7168 8192}; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --helpers $h > gpurun_out/hs_$h.json 2> gpurun_out/hs_$h.log || { tail -5 gpurun_out/hs_$h.log; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/hs_$h.json'));r=d['roofline'];print('r$r helpers $h', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step']*1e3,3), 'us/step kernel', round(r['kernel_avg_us'],3))"
done; done
