#!/bin/bash
# A/B of library variants (tools/variant.py) on the closed-loop line: the policy
# alone (NativeSAC choose_action on 65 536 obs) and both closed-loop forms, per
# variant, alternating rounds. VARIANTS="base v1 v2"; base = the in-tree library.
set -o pipefail
mkdir -p gpurun_out
for round in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARIANTS:-base}; do
    if [ "$v" = base ]; then unset SACENV_LIB; else export SACENV_LIB=$PWD/sac-agent_amd/build/libsacenv_$v.so; fi
    timeout -k 10 200 python bench.py --closed-loop --no-cpu-baseline > gpurun_out/abc_$v.json 2> gpurun_out/abc_$v.log || { tail -5 gpurun_out/abc_$v.log; exit 1; }
    unset SACENV_LIB
    python -c "import json;d=json.load(open('gpurun_out/abc_$v.json'));m=d['modes'];print('r$round $v', 'act', round(d['policy_alone_us_per_step'],2), 'us; eager', round(m['eager']['ms_per_step']*1e3,2), 'us/step; handoff', round(m['handoff']['ms_per_step']*1e3,2))"
  done
done
