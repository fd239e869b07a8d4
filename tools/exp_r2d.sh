# Llama-3-8B-shaped layer GPU test, driver-settings HTTP bench with the current tile heuristics, and an
# up-to-date c128 engine kernel table (rocprofv3 kernel trace).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -k llama3_8b -m gpu -x -q -s --timeout 200 --timeout-method thread > gpurun_out/l8b.log 2>&1 || { tail -30 gpurun_out/l8b.log; exit 1; }
grep -E "rel errors|passed|failed" gpurun_out/l8b.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_http2.json 2> gpurun_out/bench_http2.err || { tail gpurun_out/bench_http2.err; exit 1; }
tail -1 gpurun_out/bench_http2.json | cut -c1-400
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c128f -o run -- python3 bench.py --path engine --steps 100 --warmup 150 > gpurun_out/prof_c128f.log 2>&1 || { tail -20 gpurun_out/prof_c128f.log; exit 1; }
grep '^{' gpurun_out/prof_c128f.log | tail -1 | cut -c1-300
python tools/prof_summary.py gpurun_out/prof_c128f --top 30 --steps 250 > gpurun_out/prof_c128f.md
head -20 gpurun_out/prof_c128f.md
find gpurun_out/prof_c128f -name "*.db" -delete; find gpurun_out/prof_c128f -name "*kernel_trace.csv" -delete
