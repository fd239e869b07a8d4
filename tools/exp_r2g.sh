# fused dense Q|K|V for mixed-quant-type layers (large-M path) + vectorised argmax: GPU tests, engine c128
# A/B of the qkv change is implicit (previous c128 runs), driver-settings HTTP bench, batch-1.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py tests/test_kernels_gpu.py -k "llama3 or forward or argmax or sampling or engine" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/g_tests.log 2>&1 || { tail -40 gpurun_out/g_tests.log; exit 1; }
tail -1 gpurun_out/g_tests.log
timeout -k 10 300 python bench.py --path engine --steps 100 --warmup 150 > gpurun_out/g_c128.json 2> gpurun_out/g_c128.err || { tail gpurun_out/g_c128.err; exit 1; }
tail -1 gpurun_out/g_c128.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("c128", d["value"], d["ms_per_step"], d["p50_ttft_ms"], d["config"].get("dense_weight_copy_gb"))'
timeout -k 10 300 python bench.py --path engine --concurrency 1 --steps 100 --warmup 20 > gpurun_out/g_c1.json 2> gpurun_out/g_c1.err || { tail gpurun_out/g_c1.err; exit 1; }
tail -1 gpurun_out/g_c1.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("c1", d["value"], d["ms_per_step"])'
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/g_http.json 2> gpurun_out/g_http.err || { tail gpurun_out/g_http.err; exit 1; }
tail -1 gpurun_out/g_http.json | cut -c1-300
