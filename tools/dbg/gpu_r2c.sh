set -o pipefail
R=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_model_gpu.py tests/test_kernels_gpu.py tests/test_llm_worker.py tests/test_speculative.py -m gpu > $R/gpu_r2c_tests.log 2>&1 && \
timeout -k 10 400 python -u bench.py --path engine --steps 100 --warmup 20 > $R/bench_engine_c128_r2c.json 2> $R/bench_engine_c128_r2c.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/prof_c128b -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --path engine --steps 60 --warmup 10 > $R/prof_c128b.log 2>&1 && \
cd $GRAFT_REPO_ROOT && python3 tools/trace_gaps.py gpurun_out/prof_c128b > gpurun_out/prof_c128b_gaps.txt 2>&1
