set -o pipefail
R=$GRAFT_REPO_ROOT/gpurun_out
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attn_decode" -m gpu > $R/attn_tests.log 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemma.py tests/test_kv_fp8.py -m gpu >> $R/attn_tests.log 2>&1 && \
timeout -k 10 120 python tools/dbg/attn_dec_mb.py 4096 > $R/attn_mb.json && timeout -k 10 120 python tools/dbg/attn_dec_mb.py 512 >> $R/attn_mb.json
