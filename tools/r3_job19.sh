# batch-1 decode: partition size of the paged decode attention (64 default) and the in-kernel merge, engine path
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$PWD
run() { timeout -k 10 200 env "$@" python bench.py --path engine --concurrency 1 --steps 100 --warmup 20 > gpurun_out/j19.json 2> gpurun_out/j19.err || { tail -5 gpurun_out/j19.err; exit 1; }
  tail -1 gpurun_out/j19.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'"$*"'", d["value"], d["ms_per_step"])'; }
run MX_DECODE_PART_SMALL_B=64
run MX_DECODE_PART_SMALL_B=128
run MX_DECODE_PART_SMALL_B=256
run MX_DECODE_PART_SMALL_B=64 MX_ATTN_FUSED_MERGE=1
run MX_DECODE_PART_SMALL_B=256 MX_ATTN_FUSED_MERGE=1
