#!/bin/bash
# k_step / whole-step rate against envs per GPU (one MI355X): where the roofline fraction saturates
mkdir -p gpurun_out
for n in 16384 65536 131072 262144 524288; do
  timeout -k 10 300 python bench.py --envs $n --no-cpu-baseline > gpurun_out/sweep_$n.json 2> gpurun_out/sweep_$n.log || exit 1
  python -c "import json;d=json.load(open('gpurun_out/sweep_$n.json'));r=d['roofline'];print($n, round(d['value']/1e9,3), round(d['ms_per_step']*1e3,3), round(r['kernel_avg_us'],3), round(r['frac'],3))"
done
