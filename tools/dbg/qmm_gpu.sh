timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "test_qmm or llama3_8b_shapes" > gpurun_out/qmm_tests.log 2>&1 && \
SHAPES=gate_up,qkv,wo,down MS=64,128,256,512,2048 timeout -k 10 600 python -u tools/tune_qmm.py > gpurun_out/tune_qmm_v4.jsonl 2> gpurun_out/tune_qmm_v4.err
