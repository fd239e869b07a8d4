set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 500 python -u tools/tune_qmm2.py > gpurun_out/tune_qmm2_a.jsonl 2> gpurun_out/tune_qmm2_a.err || { tail -20 gpurun_out/tune_qmm2_a.err; exit 1; }
grep '"shape"' gpurun_out/tune_qmm2_a.jsonl | grep -v '"cfg"' | cut -c1-300
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/s_model_gpu.log 2>&1 || { tail -30 gpurun_out/s_model_gpu.log; exit 1; }
tail -1 gpurun_out/s_model_gpu.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/s_bench.json 2> gpurun_out/s_bench.err || { tail gpurun_out/s_bench.err; exit 1; }
tail -1 gpurun_out/s_bench.json | cut -c1-600
