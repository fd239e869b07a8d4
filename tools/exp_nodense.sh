# Driver-settings HTTP bench with the dense f16 weight copy never used (qmm at every M) vs the default,
# plus a kernel-trace of the default engine path (c128 steady state).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 env MX_DENSE_MIN_M_SWIGLU=1000000 MX_DENSE_MIN_M_NOSPLIT=1000000 MX_DENSE_MIN_M_SPLIT=1000000 \
  python bench.py --steps 20 --warmup 5 > gpurun_out/bench_nodense.json 2> gpurun_out/bench_nodense.err || exit $?
tail -1 gpurun_out/bench_nodense.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c128 -o run -- \
  python3 bench.py --path engine --steps 100 --warmup 150 > gpurun_out/prof_c128.log 2>&1 || exit $?
python tools/prof_summary.py gpurun_out/prof_c128 --top 30 --steps 100 > gpurun_out/prof_c128.md
tail -3 gpurun_out/prof_c128.log
