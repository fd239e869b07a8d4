# Split top-k sampler + fused decode-attention merge: numerics, headline bench, batch-1 engine kernel table,
# then qmm on Q4_K vs MX4F (pre-decoded scales) at the serving shapes.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_lumina2.py tests/test_sana.py -m gpu -k "sampling or attn_decode or argmax or qmv or lumina2 or gqa or sana or dwconv" -x -q --timeout 120 --timeout-method thread > gpurun_out/j8_k.log 2>&1 || { tail -30 gpurun_out/j8_k.log; exit 1; }
tail -1 gpurun_out/j8_k.log
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py tests/test_kv_fp8.py tests/test_gemma.py tests/test_speculative.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/j8_e.log 2>&1 || { tail -30 gpurun_out/j8_e.log; exit 1; }
tail -1 gpurun_out/j8_e.log
timeout -k 10 420 python bench.py --steps 20 --warmup 5 > gpurun_out/j8_bench.json 2> gpurun_out/j8_bench.err || { tail gpurun_out/j8_bench.err; exit 1; }
tail -1 gpurun_out/j8_bench.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], d["p50_ttft_ms"], json.dumps(c.get("other_phases")))'
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_j8c1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --path engine --concurrency 1 --steps 200 --warmup 50 > $GRAFT_REPO_ROOT/gpurun_out/prof_j8c1.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_j8c1.log; exit 1; }
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py gpurun_out/prof_j8c1 --top 30 --steps 250 > gpurun_out/prof_j8c1.md && head -40 gpurun_out/prof_j8c1.md
tail -1 gpurun_out/prof_j8c1.log
timeout -k 10 200 python bench.py --path engine --concurrency 1 --steps 100 --warmup 20 > gpurun_out/j8_c1.json 2>gpurun_out/j8_c1.err || { tail gpurun_out/j8_c1.err; exit 1; }
tail -1 gpurun_out/j8_c1.json
for sh in gate_up down; do
  for M in 128 2048; do
    for qt in 12 3; do
      timeout -k 10 60 python tools/prof_qmm.py --shape $sh --M $M --qt $qt --iters 20 >> gpurun_out/j8_cmp.log 2>&1 || { tail -5 gpurun_out/j8_cmp.log; exit 1; }
    done
  done
done
grep -v amdgpu.ids gpurun_out/j8_cmp.log
