set -o pipefail
R=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_model_gpu.py tests/test_kernels_gpu.py tests/test_llm_worker.py tests/test_speculative.py tests/test_moe.py -m gpu > $R/gpu_r2d_tests.log 2>&1 && \
timeout -k 10 400 python -u bench.py --path engine --steps 60 --warmup 10 > $R/bench_mixed.json 2> $R/bench_mixed.err
