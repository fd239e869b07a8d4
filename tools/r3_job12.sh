set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 120 python -u tools/dbg/rwkv_gpu.py > gpurun_out/d_rwkv1.log 2>&1; echo "rc=$?"; grep -v amdgpu.ids gpurun_out/d_rwkv1.log | tail -6
for b in 4 1,2,4; do
timeout -k 10 120 python -u tools/dbg/rwkv_gpu5.py $b > gpurun_out/d_rwkv5_$b.log 2>&1; echo "rc=$?"; grep -v amdgpu.ids gpurun_out/d_rwkv5_$b.log | tail -12
done
timeout -k 10 200 python -u -m pytest tests/test_rwkv.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/d_rwkv_pytest.log 2>&1; echo "rc=$?"; tail -3 gpurun_out/d_rwkv_pytest.log
