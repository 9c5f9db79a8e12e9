mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "mixed_segment_equals" -v --timeout 300 --timeout-method thread > gpurun_out/mixed.log 2>&1 || exit 1
timeout -k 10 300 python tools/phase_stamps.py > gpurun_out/phase.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_driver.json 2> gpurun_out/bench_driver.err || exit 1
timeout -k 10 300 python bench.py --mixed --no-cpu-baseline > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err
