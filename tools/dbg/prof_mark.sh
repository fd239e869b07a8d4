set -o pipefail
R=$GRAFT_REPO_ROOT/gpurun_out
cd /tmp && export TMPDIR=/tmp
export MX_ROCTX=1
timeout -k 10 500 rocprofv3 --kernel-trace --marker-trace -d $R/prof_mark -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --path engine --steps 40 --warmup 10 > $R/prof_mark.log 2>&1 && \
cd $GRAFT_REPO_ROOT && python3 tools/dbg/hip_gaps.py gpurun_out/prof_mark > gpurun_out/prof_mark_gaps.txt 2>&1; rm -rf gpurun_out/prof_mark
