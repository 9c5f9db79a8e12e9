#!/bin/bash
# refill + closed-loop changes: parity tests, then the bench lines and ablations (round 4)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_bench_path_gpu.py tests/test_segment_gpu.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/par.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --closed-loop > gpurun_out/bench_closed.json 2> gpurun_out/bench_closed.err || exit 1
VARIANTS="base abl_norow abl_nostore abl_nocnt abl_norestart" ROUNDS=2 bash tools/ab_r04.sh > gpurun_out/ab2.txt 2>&1
