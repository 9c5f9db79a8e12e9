#!/bin/bash
# GPU tests, then A/B lines: the in-tree library against variants built by
# tools/variant.py (VARIANTS_SEG for the default bench line, VARIANTS_STEP for
# --launch step). Each GPU step under its own time limit; the first failure ends it.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
[ -n "$VARIANTS_SEG" ] && { VARIANTS="$VARIANTS_SEG" ROUNDS=${ROUNDS:-3} BENCH_ARGS="--no-cpu-baseline" bash tools/ab_lib.sh || exit 1; }
[ -n "$VARIANTS_STEP" ] && { VARIANTS="$VARIANTS_STEP" ROUNDS=2 BENCH_ARGS="--launch step --no-cpu-baseline --steps 1024 --warmup 256" bash tools/ab_lib.sh || exit 1; }
echo ab_step done
