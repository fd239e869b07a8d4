set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_moe.py tests/test_hf_loader.py tests/test_kernels_gpu.py -m gpu > gpurun_out/gpu_r2b_tests.log 2>&1 && \
timeout -k 10 400 python -u bench.py --path engine --steps 100 --warmup 20 > gpurun_out/bench_engine_c128_r2b.json 2> gpurun_out/bench_engine_c128_r2b.err
