# c128 engine path: decode-attention partition 512 (default) vs 1024 (one partition at these lengths: no reduce)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$PWD
run() { timeout -k 10 300 env "$@" python bench.py --path engine --concurrency 128 --steps 100 --warmup 20 > gpurun_out/j24.json 2> gpurun_out/j24.err || { tail -5 gpurun_out/j24.err; exit 1; }
  tail -1 gpurun_out/j24.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'"$*"'", d["value"], d["ms_per_step"])'; }
run MX_DECODE_PART_LARGE_B=512
run MX_DECODE_PART_LARGE_B=1024
run MX_DECODE_PART_LARGE_B=512
run MX_DECODE_PART_LARGE_B=1024
