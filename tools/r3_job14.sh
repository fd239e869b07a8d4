set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$PWD
for m in keepgraphs rocblas q8 none; do
timeout -k 10 120 python -u tools/dbg/rwkv_gpu7.py $m > gpurun_out/f_rwkv7_$m.log 2>&1; echo "rc=$?"; grep -v amdgpu.ids gpurun_out/f_rwkv7_$m.log | tail -6
done
