# overlap depth 1 vs 2 on the driver-settings HTTP bench, two runs each (run-to-run noise)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$PWD
for r in 1 2; do for d in 1 2; do
  timeout -k 10 400 env MX_OVERLAP_DEPTH=$d python bench.py --steps 20 --warmup 5 > gpurun_out/m_d${d}_r$r.json 2> gpurun_out/m_d${d}_r$r.err || { tail gpurun_out/m_d${d}_r$r.err; exit 1; }
  tail -1 gpurun_out/m_d${d}_r$r.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("depth='$d' run='$r'", d["value"], d["ms_per_step"], d["p50_ttft_ms"], d["config"]["p99_itl_ms"])'
done; done
