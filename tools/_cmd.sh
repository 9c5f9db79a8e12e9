set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
SACENV_BENCH_ONE_DEVICE=1 SACENV_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 300 --warmup 100 --envs 8192 > gpurun_out/rehearse2.json 2> gpurun_out/rehearse2.log || { tail -30 gpurun_out/rehearse2.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/rehearse2.json'));print('dp2 rehearsal', round(d['value']/1e6,1), 'M/s', d['config']['collective'])"
timeout -k 10 300 python bench.py --steps 1000 --warmup 200 --no-cpu-baseline > gpurun_out/b.json 2> gpurun_out/b.log || exit 1
python -c "import json;d=json.load(open('gpurun_out/b.json'));print('n1', round(d['value']/1e9,3), 'G/s')"
