set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$PWD
for m in plain rocblas prime_mm; do
timeout -k 10 120 python -u tools/dbg/rwkv_gpu4.py $m > gpurun_out/c_rwkv_$m.log 2>&1; echo "rc=$?"; grep -v amdgpu.ids gpurun_out/c_rwkv_$m.log | tail -2
done
timeout -k 10 300 python -u tools/tune_qmm_ws.py --shapes gate_up --M 128 --cfgs 441412,41411 --dbg 15,31,63,47,16,32 > gpurun_out/c_dbg.jsonl 2> gpurun_out/c_dbg.err || { tail -5 gpurun_out/c_dbg.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/c_dbg.jsonl'):
    d=json.loads(l); print(d['shape'],d['M'],'qmm',d['qmm_us'])
    for w in d['ws']: print('   ',{k:v for k,v in w.items() if k!='tflops'})
"
