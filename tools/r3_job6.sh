# Fast-sampler + qmm8 tests, headline bench, diffusion (MMDiT-X, GGUF-quantised SD3.5-medium) GPU tests,
# a batch-1 engine kernel table, then the qmm counter passes.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/test_diffusion.py tests/test_sd_gguf_quant.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/j6_diff.log 2>&1 || { tail -30 gpurun_out/j6_diff.log; exit 1; }
tail -1 gpurun_out/j6_diff.log
timeout -k 10 300 python -u -m pytest tests/test_quant_formats.py tests/test_kernels_gpu.py -m gpu -k "mxf or carried or qmm or qmv_t32 or qmatmul or relative_bias or rope" -x -q --timeout 120 --timeout-method thread > gpurun_out/j6_mxf.log 2>&1 || { tail -30 gpurun_out/j6_mxf.log; exit 1; }
tail -1 gpurun_out/j6_mxf.log
timeout -k 10 300 python -u -m pytest tests/test_tts.py tests/test_bark.py tests/test_musicgen.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/j6_audio.log 2>&1 || { tail -30 gpurun_out/j6_audio.log; exit 1; }
tail -1 gpurun_out/j6_audio.log
timeout -k 10 420 python bench.py --steps 20 --warmup 5 > gpurun_out/j6_bench.json 2> gpurun_out/j6_bench.err || { tail gpurun_out/j6_bench.err; exit 1; }
tail -1 gpurun_out/j6_bench.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], d["p50_ttft_ms"], c.get("dense_weight_copy_gb"), json.dumps(c.get("other_phases")))'
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_j6c1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --path engine --concurrency 1 --steps 200 --warmup 50 > $GRAFT_REPO_ROOT/gpurun_out/prof_j6c1.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_j6c1.log; exit 1; }
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py gpurun_out/prof_j6c1 --top 30 --steps 250 > gpurun_out/prof_j6c1.md && head -40 gpurun_out/prof_j6c1.md
tail -1 gpurun_out/prof_j6c1.log
timeout -k 10 300 env MX_QMM8=1 python -u -m pytest tests/test_qmm8_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/j6_q8.log 2>&1 || { tail -30 gpurun_out/j6_q8.log; exit 1; }
tail -1 gpurun_out/j6_q8.log
bash tools/pmc_qmm_r3.sh
