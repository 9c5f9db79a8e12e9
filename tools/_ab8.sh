set -o pipefail
export TMPDIR=/tmp
VARIANTS="base fmaplain expocml" BENCH_ARGS="--steps 2048 --warmup 512 --no-cpu-baseline" bash tools/ab.sh || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/pytest_gpu.log
