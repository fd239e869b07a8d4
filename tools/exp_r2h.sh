# decode attention split-K merge in the last-arriving workgroup (no separate merge kernel): kernel + model
# GPU tests, engine c1 / c128 A/B (MX_ATTN_FUSED_MERGE=0 vs 1), driver-settings HTTP bench.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_speculative.py tests/test_kv_fp8.py -k "attn or forward or engine or llama3 or gpu" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/h_tests.log 2>&1 || { tail -40 gpurun_out/h_tests.log; exit 1; }
tail -1 gpurun_out/h_tests.log
for c in 1 128; do for f in 0 1; do
  w=20; [ $c = 128 ] && w=150
  timeout -k 10 300 env MX_ATTN_FUSED_MERGE=$f python bench.py --path engine --concurrency $c --steps 100 --warmup $w > gpurun_out/h_c${c}_m$f.json 2> gpurun_out/h_c${c}_m$f.err || { tail gpurun_out/h_c${c}_m$f.err; exit 1; }
  tail -1 gpurun_out/h_c${c}_m$f.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("c='$c' merge='$f'", d["value"], d["ms_per_step"], d["p50_ttft_ms"])'
done; done
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/h_http.json 2> gpurun_out/h_http.err || { tail gpurun_out/h_http.err; exit 1; }
tail -1 gpurun_out/h_http.json | cut -c1-300
