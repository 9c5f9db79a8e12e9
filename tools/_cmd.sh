set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
SACENV_BENCH_ONE_DEVICE=1 SACENV_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 300 --warmup 100 --envs 8192 > gpurun_out/rehearse2.json 2> gpurun_out/rehearse2.log || { tail -30 gpurun_out/rehearse2.log; exit 1; }
cat gpurun_out/rehearse2.json
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.log || exit 1
cat gpurun_out/bench_default.json
