#!/bin/bash
# The N>1 bench path rehearsed on one GPU: 2 ranks over gloo sharing the device
# (the driver's 8-GPU run uses RCCL, one rank per GPU), then the bench GPU tests.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_bench_gpu.py -x -q --timeout 240 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_bench_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_bench_gpu.log; [ $rc -eq 0 ] || exit $rc
for pe in ${POOL_EVERY:-128}; do
  SACENV_BENCH_BACKEND=gloo SACENV_BENCH_ONE_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29500 + pe)) bench.py --gpus 2 \
    --envs 65536 --pool-every $pe --steps 256 --warmup 128 > gpurun_out/rehearse_pe$pe.json \
    2> gpurun_out/rehearse_pe$pe.log || { tail -20 gpurun_out/rehearse_pe$pe.log; exit 1; }
  tail -1 gpurun_out/rehearse_pe$pe.json | python -c "import json,sys;d=json.loads(sys.stdin.read());p=d['pooling'];print('pool_every', p['pool_every'], round(d['value']/1e9,3), 'G/s; no exchange', round(p['no_exchange']['value']/1e9,3), 'G/s')"
done
