set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_default.json 2> gpurun_out/bench_default.log || exit 1
python -c "import json;d=json.load(open('gpurun_out/bench_default.json'));print('N1', d['value']/1e9, d['roofline']['kernel_avg_us'], d['roofline']['step_us_incl_refill'])"
SACENV_BENCH_BACKEND=gloo SACENV_BENCH_ONE_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 256 --warmup 128 > gpurun_out/rehearse_dp2.json 2> gpurun_out/rehearse_dp2.log; echo "dp2 rc=$?"; tail -c 1500 gpurun_out/rehearse_dp2.json
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters.txt 2>&1; echo "list rc=$?"
