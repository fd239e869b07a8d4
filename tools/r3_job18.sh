# step token budget A/B on the driver-settings HTTP bench: 2048 (bench default so far), 512 (the reference's
# default NBatch, core/backend/options.go:76-79), 256
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$PWD
for b in 512 256 2048; do
timeout -k 10 420 python bench.py --gpus 1 --steps 20 --warmup 5 --max-batched-tokens $b > gpurun_out/j18_b$b.json 2> gpurun_out/j18_b$b.err || { tail gpurun_out/j18_b$b.err; exit 1; }
tail -1 gpurun_out/j18_b$b.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print('$b', d["value"], d["ms_per_step"], d["p50_ttft_ms"], d["p99_ttft_ms"], json.dumps(d["config"].get("other_phases")))'
done
