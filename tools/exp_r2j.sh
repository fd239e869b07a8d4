# batch-1 decode-attention partition length (64 = 5 partials + merge kernel at ~300-token contexts, 512 =
# one partition, no merge), and the driver-settings HTTP bench with the current defaults.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$PWD
for p in 64 256 512; do
  timeout -k 10 300 env MX_DECODE_PART_SMALL_B=$p python bench.py --path engine --concurrency 1 --steps 100 --warmup 20 > gpurun_out/j_c1_p$p.json 2> gpurun_out/j_c1_p$p.err || { tail gpurun_out/j_c1_p$p.err; exit 1; }
  tail -1 gpurun_out/j_c1_p$p.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("c1 part='$p'", d["value"], d["ms_per_step"])'
done
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/j_http.json 2> gpurun_out/j_http.err || { tail gpurun_out/j_http.err; exit 1; }
tail -1 gpurun_out/j_http.json | cut -c1-300
