set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$PWD
for m in f32 rocblas q8; do
timeout -k 10 120 python -u tools/dbg/rwkv_gpu3.py $m > gpurun_out/b_rwkv_$m.log 2>&1; echo "rc=$?"; grep -v amdgpu.ids gpurun_out/b_rwkv_$m.log | tail -4
done
timeout -k 10 200 python -u tools/tune_qmm_ws.py --shapes gate_up --M 128 --cfgs 41411,22211,22212 --dbg 1,2,3,4,8,12,15,7,11 > gpurun_out/b_dbg.jsonl 2> gpurun_out/b_dbg.err || { tail -5 gpurun_out/b_dbg.err; exit 1; }
cat gpurun_out/b_dbg.jsonl
