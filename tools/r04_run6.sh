#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_bench_path_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/par6.log 2>&1 || exit 1
bash tools/ktrace.sh > gpurun_out/kt.txt 2>&1
