# A/B of the GEMM paths on the driver-settings HTTP bench (now: BPE tokenizer + reference sampling phase,
# greedy second phase) and a c128 engine kernel table for the default path.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$PWD
for v in "q8:MX_QMM8=1" "f16:MX_QMM8=0" "dense:MX_QMM8=0 MX_DENSE_CACHE=1"; do
  n=${v%%:*}; e=${v#*:}
  timeout -k 10 420 env $e python bench.py --steps 20 --warmup 5 > gpurun_out/j4_$n.json 2> gpurun_out/j4_$n.err || { tail gpurun_out/j4_$n.err; exit 1; }
  tail -1 gpurun_out/j4_$n.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print("'$n'", d["value"], d["ms_per_step"], d["p50_ttft_ms"], c.get("dense_weight_copy_gb"), json.dumps(c.get("other_phases")))'
done
cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_j4 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --path engine --steps 100 --warmup 150 > $GRAFT_REPO_ROOT/gpurun_out/prof_j4.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_j4.log; exit 1; }
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py gpurun_out/prof_j4 --top 40 --steps 250 > gpurun_out/prof_j4.md && head -50 gpurun_out/prof_j4.md
