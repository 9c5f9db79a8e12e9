set -o pipefail
VARIANTS="base sc1 nt kin" BENCH_ARGS="--steps 2048 --warmup 512 --no-cpu-baseline" bash tools/ab.sh || exit 1
SACENV_LIB=$PWD/sac-agent_amd/build/libsacenv_kin.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "seeded or autoreset or full_size or rollout or recorded" > gpurun_out/kin_parity.log 2>&1; echo "kin parity rc=$?"; tail -3 gpurun_out/kin_parity.log
