# Re-verify after a container rebuild: smoke, full GPU suite, driver-settings bench, overlap-depth A/B,
# no-dense-copy A/B, batch-1. Stops at the first failure (every GPU step has its own time limit).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log | cut -c1-200
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -rf > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_http.json 2> gpurun_out/bench_http.err || { tail gpurun_out/bench_http.err; exit 1; }
tail -1 gpurun_out/bench_http.json | cut -c1-600
for d in 1 2; do
  timeout -k 10 300 env MX_OVERLAP_DEPTH=$d python bench.py --path engine --steps 100 --warmup 150 > gpurun_out/depth_$d.json 2> gpurun_out/depth_$d.err || { tail gpurun_out/depth_$d.err; exit 1; }
  tail -1 gpurun_out/depth_$d.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("engine depth='$d'", d["value"], d["ms_per_step"], d["p50_ttft_ms"], d["config"].get("host_ms_per_step"))'
done
timeout -k 10 300 env MX_DENSE_MIN_M_SWIGLU=1000000 MX_DENSE_MIN_M_NOSPLIT=1000000 MX_DENSE_MIN_M_SPLIT=1000000 \
  python bench.py --path engine --steps 100 --warmup 150 > gpurun_out/nodense.json 2> gpurun_out/nodense.err || { tail gpurun_out/nodense.err; exit 1; }
tail -1 gpurun_out/nodense.json | cut -c1-300
timeout -k 10 300 python bench.py --path engine --concurrency 1 --steps 100 --warmup 20 > gpurun_out/c1.json 2> gpurun_out/c1.err || { tail gpurun_out/c1.err; exit 1; }
tail -1 gpurun_out/c1.json | cut -c1-300
