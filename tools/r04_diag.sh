#!/bin/bash
export DIAG_N=8192 DIAG_K=128
for v in base nopad normalpad; do
  if [ "$v" = base ]; then unset SACENV_LIB; else export SACENV_LIB=$PWD/sac-agent_amd/build/libsacenv_$v.so; fi
  echo "== $v"; timeout -k 10 120 python tools/diag_closed_loop.py 2>&1 | grep -v amdgpu.ids || exit 1
done
