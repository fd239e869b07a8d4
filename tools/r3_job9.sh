set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 200 python -u tools/dbg/rwkv_gpu.py > gpurun_out/a_rwkv.log 2>&1; echo "rwkv rc=$?"; grep -v amdgpu.ids gpurun_out/a_rwkv.log | tail -8
timeout -k 10 300 python -u tools/tune_qmm_ws.py --shapes gate_up,qkv,wo,down --M 128,256 > gpurun_out/a_ws.jsonl 2> gpurun_out/a_ws.err || { tail -20 gpurun_out/a_ws.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/a_ws.jsonl'):
    d=json.loads(l); b=d.get('best',{}); print(d['shape'],d['M'],'qmm',d['qmm_us'],'best',b.get('cfg'),b.get('splits'),b.get('us'),'x',d.get('speedup'),'errs',max([w.get('rel_err',0) for w in d['ws']]))
"
