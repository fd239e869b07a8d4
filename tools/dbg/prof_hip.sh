set -o pipefail
R=$GRAFT_REPO_ROOT/gpurun_out
cd /tmp && export TMPDIR=/tmp
export MX_ROCTX=1
timeout -k 10 500 rocprofv3 --kernel-trace --hip-runtime-trace --marker-trace -d $R/prof_hip -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --path engine --steps 40 --warmup 10 > $R/prof_hip.log 2>&1 && \
cd $GRAFT_REPO_ROOT && python3 tools/dbg/hip_gaps.py gpurun_out/prof_hip > gpurun_out/prof_hip_gaps.txt 2>&1; rm -rf gpurun_out/prof_hip
