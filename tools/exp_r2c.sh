# small-M qmm tiles (two workgroups per CU) A/B on the engine at c32 / c64, engine GPU tests, and the
# SD3 /v1/images/generations HTTP bench (BASELINE config #5, 1 GPU).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/model_gpu.log 2>&1 || { tail -30 gpurun_out/model_gpu.log; exit 1; }
tail -1 gpurun_out/model_gpu.log
for c in 32 64; do for o in 0 1; do
  timeout -k 10 300 env MX_QMM_OCC=$o python bench.py --path engine --concurrency $c --steps 100 --warmup 60 > gpurun_out/c${c}_occ$o.json 2> gpurun_out/c${c}_occ$o.err || { tail gpurun_out/c${c}_occ$o.err; exit 1; }
  tail -1 gpurun_out/c${c}_occ$o.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("c='$c' occ='$o'", d["value"], d["ms_per_step"], d["p50_ttft_ms"], d["config"].get("dense_weight_copy_gb"))'
done; done
timeout -k 10 600 python -u tools/bench_images_http.py --gpus 1 --size 1024 --steps 28 --images 6 --concurrency 2 > gpurun_out/images_http.json 2> gpurun_out/images_http.err || { tail -20 gpurun_out/images_http.err; exit 1; }
tail -1 gpurun_out/images_http.json
