#!/bin/bash
# Round-end check on one GPU box: parity tests, smoke(), the bench configs,
# and a rocprofv3 kernel-trace summary of the default bench line.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_round.sh || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o run --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.log || exit 1
find gpurun_out/prof_final -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} gpurun_out/final_kernel_stats.csv
echo done
