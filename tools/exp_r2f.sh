# fused-input decode GEMVs (RMSNorm / q8 quantisation in the qmv prologue): kernel + model GPU tests,
# batch-1 and batch-4 engine A/B (MX_QMV_FUSE=0 vs 1), driver-settings HTTP bench.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_gemma.py -k "qmv or forward or engine or llama3 or gpu" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/fuse_tests.log 2>&1 || { tail -40 gpurun_out/fuse_tests.log; exit 1; }
tail -1 gpurun_out/fuse_tests.log
for c in 1 4; do for f in 0 1; do
  timeout -k 10 300 env MX_QMV_FUSE=$f python bench.py --path engine --concurrency $c --steps 100 --warmup 20 > gpurun_out/c${c}_fuse$f.json 2> gpurun_out/c${c}_fuse$f.err || { tail gpurun_out/c${c}_fuse$f.err; exit 1; }
  tail -1 gpurun_out/c${c}_fuse$f.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("c='$c' fuse='$f'", d["value"], d["ms_per_step"])'
done; done
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_http3.json 2> gpurun_out/bench_http3.err || { tail gpurun_out/bench_http3.err; exit 1; }
tail -1 gpurun_out/bench_http3.json | cut -c1-300
