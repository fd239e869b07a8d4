# decode-attention partition length at c128 (256 vs 512: no merge kernel for <= 512-token contexts), then the
# full GPU suite + smoke after this session's kernel changes.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$PWD
for p in 256 512; do
  timeout -k 10 300 env MX_DECODE_PART_LARGE_B=$p python bench.py --path engine --steps 100 --warmup 150 > gpurun_out/i_c128_p$p.json 2> gpurun_out/i_c128_p$p.err || { tail gpurun_out/i_c128_p$p.err; exit 1; }
  tail -1 gpurun_out/i_c128_p$p.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("c128 part='$p'", d["value"], d["ms_per_step"], d["p50_ttft_ms"])'
done
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/i_smoke.log 2>&1 || { tail -20 gpurun_out/i_smoke.log; exit 1; }
tail -1 gpurun_out/i_smoke.log | cut -c1-150
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -rf > gpurun_out/i_gpu_suite.log 2>&1 || { tail -30 gpurun_out/i_gpu_suite.log; exit 1; }
tail -2 gpurun_out/i_gpu_suite.log
