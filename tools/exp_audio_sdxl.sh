# GPU: diffusion kernel tests, SDXL 1024^2 step time on the MFMA conv kernel vs MIOpen, audio model timings,
# then the one-shot IPC all-reduce multi-process test (last: it is the one that could stall).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_diffusion.py tests/test_unet.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/diff_tests.log 2>&1 || { tail -30 gpurun_out/diff_tests.log; exit 1; }
tail -2 gpurun_out/diff_tests.log
timeout -k 10 300 python tools/bench_sdxl.py --size 1024 --steps 20 > gpurun_out/sdxl.jsonl 2> gpurun_out/sdxl.err || { tail gpurun_out/sdxl.err; exit 1; }
timeout -k 10 300 env MX_CONV=miopen python tools/bench_sdxl.py --size 1024 --steps 20 >> gpurun_out/sdxl.jsonl 2>> gpurun_out/sdxl.err || exit $?
cat gpurun_out/sdxl.jsonl
timeout -k 10 300 python tools/bench_audio.py > gpurun_out/audio.jsonl 2> gpurun_out/audio.err || { tail gpurun_out/audio.err; exit 1; }
cat gpurun_out/audio.jsonl
timeout -k 10 300 python -u -m pytest tests/test_custom_ar.py -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/ar_tests.log 2>&1; rc=$?; tail -30 gpurun_out/ar_tests.log; exit $rc
