# A/B of the overlap pipeline depth (engine/engine.py overlap_depth) + GPU engine tests.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/model_gpu.log 2>&1 || { tail -30 gpurun_out/model_gpu.log; exit 1; }
tail -1 gpurun_out/model_gpu.log
for d in 1 2 3; do
  timeout -k 10 300 env MX_OVERLAP_DEPTH=$d python bench.py --path engine --steps 100 --warmup 150 > gpurun_out/depth_$d.json 2> gpurun_out/depth_$d.err || { tail gpurun_out/depth_$d.err; exit 1; }
  tail -1 gpurun_out/depth_$d.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("engine depth='$d'", d["value"], d["ms_per_step"], d["p50_ttft_ms"], d["config"]["host_ms_per_step"])'
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/depth_http.json 2> gpurun_out/depth_http.err || exit $?
tail -1 gpurun_out/depth_http.json
timeout -k 10 300 python bench.py --path engine --concurrency 1 --steps 100 --warmup 20 > gpurun_out/depth_c1.json 2> gpurun_out/depth_c1.err || exit $?
tail -1 gpurun_out/depth_c1.json | cut -c1-400
