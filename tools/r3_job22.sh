# c128 engine path, default GEMM path (qmm.hip f16, no dense copy), reference sampling: kernel table
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$PWD
cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_j22 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --path engine --concurrency 128 --steps 100 --warmup 20 > $GRAFT_REPO_ROOT/gpurun_out/prof_j22.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_j22.log; exit 1; }
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py gpurun_out/prof_j22 --top 32 --steps 120 > gpurun_out/prof_j22.md && head -40 gpurun_out/prof_j22.md
tail -1 gpurun_out/prof_j22.log | cut -c1-300
