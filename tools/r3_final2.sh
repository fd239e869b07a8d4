# final round-3 check on the committed tree: smoke + full GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3g_smoke.log 2>&1 || { tail -20 gpurun_out/r3g_smoke.log; exit 1; }
tail -1 gpurun_out/r3g_smoke.log | cut -c1-160
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -rf > gpurun_out/r3g_gpu_suite.log 2>&1 || { tail -30 gpurun_out/r3g_gpu_suite.log; exit 1; }
tail -1 gpurun_out/r3g_gpu_suite.log
