set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -m gpu -k "test_qmm and Q4_K" -q --timeout 120 --timeout-method thread > gpurun_out/dbg_q4k.log 2>&1; tail -3 gpurun_out/dbg_q4k.log
timeout -k 10 200 python -u tools/dbg_mxf.py > gpurun_out/dbg_mxf.log 2>&1; tail -40 gpurun_out/dbg_mxf.log
