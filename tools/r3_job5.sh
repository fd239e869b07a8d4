set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "sampling or penalties or qmv_t32" -x -q --timeout 120 --timeout-method thread > gpurun_out/j5_tests.log 2>&1 || { tail -30 gpurun_out/j5_tests.log; exit 1; }
tail -1 gpurun_out/j5_tests.log
timeout -k 10 300 env MX_QMM8=1 python -u -m pytest tests/test_qmm8_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/j5_q8.log 2>&1 || { tail -30 gpurun_out/j5_q8.log; exit 1; }
tail -1 gpurun_out/j5_q8.log
timeout -k 10 420 python bench.py --steps 20 --warmup 5 > gpurun_out/j5_bench.json 2> gpurun_out/j5_bench.err || { tail gpurun_out/j5_bench.err; exit 1; }
tail -1 gpurun_out/j5_bench.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], d["p50_ttft_ms"], c.get("dense_weight_copy_gb"), json.dumps(c.get("other_phases")))'
bash tools/pmc_qmm_r3.sh
