# qmm two-workgroups-per-CU (half-LDS ring) A/B: GPU correctness for every config, then the tile sweep
# on the Llama-3-8B projections (one JSON line per shape x M), plus the new SVD GPU tests.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "test_qmm" tests/test_svd.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/qmm_occ_tests.log 2>&1 || { tail -30 gpurun_out/qmm_occ_tests.log; exit 1; }
tail -1 gpurun_out/qmm_occ_tests.log
timeout -k 10 600 env SHAPES=gate_up,qkv,wo,down MS=64,128,192,256,512,2048 python -u tools/tune_qmm.py > gpurun_out/tune_qmm_occ.jsonl 2> gpurun_out/tune_qmm_occ.err || { tail gpurun_out/tune_qmm_occ.err; exit 1; }
python tools/sum_tune.py gpurun_out/tune_qmm_occ.jsonl 2>/dev/null || cut -c1-260 gpurun_out/tune_qmm_occ.jsonl
