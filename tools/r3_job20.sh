# batch-1 engine path with reference sampling: kernel table
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$PWD
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_j20 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --path engine --concurrency 1 --steps 200 --warmup 50 > $GRAFT_REPO_ROOT/gpurun_out/prof_j20.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_j20.log; exit 1; }
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py gpurun_out/prof_j20 --top 30 --steps 250 > gpurun_out/prof_j20.md && head -36 gpurun_out/prof_j20.md
tail -1 gpurun_out/prof_j20.log | cut -c1-200
