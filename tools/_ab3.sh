set -o pipefail
VARIANTS="base obsplain recplain sinpoly" BENCH_ARGS="--steps 2048 --warmup 512 --no-cpu-baseline" bash tools/ab.sh || exit 1
SACENV_LIB=$PWD/sac-agent_amd/build/libsacenv_sinpoly.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "seeded or autoreset or full_size or rollout or recorded" > gpurun_out/sinpoly_parity.log 2>&1; echo "sinpoly parity rc=$?"; tail -3 gpurun_out/sinpoly_parity.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
