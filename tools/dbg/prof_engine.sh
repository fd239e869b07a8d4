set -o pipefail
R=$GRAFT_REPO_ROOT/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/prof_c128 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --path engine --steps 60 --warmup 10 > $R/prof_c128.log 2>&1 && \
cd $GRAFT_REPO_ROOT && python3 tools/trace_gaps.py gpurun_out/prof_c128 > gpurun_out/prof_c128_gaps.txt 2>&1 && python3 tools/prof_summary.py gpurun_out/prof_c128 > gpurun_out/prof_c128_summary.txt 2>&1
rm -f gpurun_out/prof_c128/run_kernel_trace.csv
