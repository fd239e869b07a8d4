# batch-1 decode: kernel table + idle gaps (rocprofv3 kernel trace)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c1 -o run -- python3 bench.py --path engine --concurrency 1 --steps 200 --warmup 20 > gpurun_out/prof_c1.log 2>&1 || { tail -20 gpurun_out/prof_c1.log; exit 1; }
grep '^{' gpurun_out/prof_c1.log | tail -1 | cut -c1-300
python tools/prof_summary.py gpurun_out/prof_c1 --top 25 --steps 220 > gpurun_out/prof_c1.md
python tools/trace_gaps.py gpurun_out/prof_c1 > gpurun_out/prof_c1_gaps.txt 2>&1 || true
cat gpurun_out/prof_c1.md; head -20 gpurun_out/prof_c1_gaps.txt
find gpurun_out/prof_c1 -name "*.db" -delete; find gpurun_out/prof_c1 -name "*kernel_trace.csv" -delete
