#!/bin/bash
# k_need_masks / k_refill / k_refill_fit / k_rollout medians per library variant (tools/ktrace.sh each)
set -o pipefail
for v in ${VARIANTS:-base}; do
  rm -rf gpurun_out/kt
  if [ "$v" = base ]; then unset SACENV_LIB; else export SACENV_LIB=$PWD/sac-agent_amd/build/libsacenv_$v.so; fi
  bash tools/ktrace.sh > gpurun_out/kt_$v.txt || exit 1
  unset SACENV_LIB
  echo "== $v"; grep -E "k_need|k_refill|k_rollout " gpurun_out/kt_$v.txt
done
