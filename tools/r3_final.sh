# round-3 rehearsal: RWKV fix check, smoke, full GPU suite, driver-style bench (N=1, steps 20, warmup 5)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 120 python -u tools/dbg/rwkv_gpu7.py none > gpurun_out/r3f_rwkv7.log 2>&1 || { tail -5 gpurun_out/r3f_rwkv7.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r3f_rwkv7.log | tail -4
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3f_smoke.log 2>&1 || { tail -20 gpurun_out/r3f_smoke.log; exit 1; }
tail -1 gpurun_out/r3f_smoke.log | cut -c1-160
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -rf > gpurun_out/r3f_gpu_suite.log 2>&1 || { tail -30 gpurun_out/r3f_gpu_suite.log; exit 1; }
tail -1 gpurun_out/r3f_gpu_suite.log
timeout -k 10 420 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3f_bench.json 2> gpurun_out/r3f_bench.err || { tail gpurun_out/r3f_bench.err; exit 1; }
tail -1 gpurun_out/r3f_bench.json | cut -c1-700
