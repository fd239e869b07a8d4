# GPU suite + driver-style bench (N=1, steps 20, warmup 5); stops at the first failure
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s_smoke.log 2>&1 || { tail -20 gpurun_out/s_smoke.log; exit 1; }
tail -1 gpurun_out/s_smoke.log | cut -c1-120
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -rf ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/s_gpu_suite.log 2>&1 || { tail -30 gpurun_out/s_gpu_suite.log; exit 1; }
tail -1 gpurun_out/s_gpu_suite.log
if [ -z "$NO_BENCH" ]; then
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/s_bench.json 2> gpurun_out/s_bench.err || { tail gpurun_out/s_bench.err; exit 1; }
tail -1 gpurun_out/s_bench.json | cut -c1-600
fi
