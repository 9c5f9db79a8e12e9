#!/bin/bash
# closed-loop tests + bench line, then the ablation A/B (round 4)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_segment_gpu.py -v -s --timeout 300 --timeout-method thread > gpurun_out/seg.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --closed-loop > gpurun_out/bench_closed.json 2> gpurun_out/bench_closed.err || exit 1
VARIANTS="base abl_norow abl_nostore abl_nocnt abl_norestart" ROUNDS=2 bash tools/ab_r04.sh > gpurun_out/ab2.txt 2>&1
