# A/B of the serving-loop GC policy (engine/engine.py gc_tune) on the engine and HTTP benches.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for g in 0 1; do
  timeout -k 10 300 env MX_GC_TUNE=$g python bench.py --path engine --steps 100 --warmup 150 > gpurun_out/gc_eng_$g.json 2> gpurun_out/gc_eng_$g.err || exit $?
  tail -1 gpurun_out/gc_eng_$g.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("engine gc_tune='$g'", d["value"], d["ms_per_step"], d["config"]["host_gc"], d["config"]["host_ms_per_step"])'
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/gc_http.json 2> gpurun_out/gc_http.err || exit $?
tail -1 gpurun_out/gc_http.json
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c1 -o run -- \
  python3 bench.py --path engine --concurrency 1 --steps 200 --warmup 50 > gpurun_out/prof_c1.log 2>&1 || exit $?
python tools/prof_summary.py gpurun_out/prof_c1 --top 25 --steps 200 > gpurun_out/prof_c1.md
grep '^{' gpurun_out/prof_c1.log | tail -1
