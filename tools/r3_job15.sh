set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 200 python -u tools/dbg/rwkv_gpu8.py > gpurun_out/g_rwkv8.log 2>&1; echo "rc=$?"; grep -v amdgpu.ids gpurun_out/g_rwkv8.log | tail -22
