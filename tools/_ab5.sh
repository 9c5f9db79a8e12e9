set -o pipefail
export TMPDIR=/tmp
VARIANTS="base ocmlsc" BENCH_ARGS="--steps 2048 --warmup 512 --no-cpu-baseline" bash tools/ab.sh || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; echo "parity rc=$?"; tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python tools/stamps.py --rebuild > gpurun_out/stamps_full.txt 2>&1; echo "stamps rc=$?"; cat gpurun_out/stamps_full.txt | tail -12
STAMP_DEFINES=-DSACENV_STAMPS_LIGHT STAMP_LIB=libsacenv_stampsl.so timeout -k 10 300 python tools/stamps.py --rebuild > gpurun_out/stamps_light.txt 2>&1; echo "stampsl rc=$?"; tail -8 gpurun_out/stamps_light.txt
