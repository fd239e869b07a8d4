set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$PWD
for m in plain gc gc_empty keep; do
timeout -k 10 120 python -u tools/dbg/rwkv_gpu6.py $m > gpurun_out/e_rwkv6_$m.log 2>&1; echo "rc=$?"; grep -v amdgpu.ids gpurun_out/e_rwkv6_$m.log | tail -3
done
