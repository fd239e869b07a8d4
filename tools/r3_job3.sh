set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/test_qmm8_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/q8_tests.log 2>&1 || { tail -40 gpurun_out/q8_tests.log; exit 1; }
tail -2 gpurun_out/q8_tests.log
timeout -k 10 400 python -u tools/tune_qmm8.py > gpurun_out/tune_qmm8_a.jsonl 2> gpurun_out/tune_qmm8_a.err || { tail -20 gpurun_out/tune_qmm8_a.err; exit 1; }
grep '"shape"' gpurun_out/tune_qmm8_a.jsonl | grep -v '"cfg"' | cut -c1-300
