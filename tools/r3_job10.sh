set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$PWD
for m in f32 q8; do
timeout -k 10 120 python -u tools/dbg/rwkv_gpu3.py $m > gpurun_out/b_rwkv_$m.log 2>&1; echo "rc=$?"; grep -v amdgpu.ids gpurun_out/b_rwkv_$m.log | tail -4
done
timeout -k 10 300 python -u tools/tune_qmm_ws.py --shapes gate_up --M 128,256 --cfgs 41411,441412,242412,241821,422212 --dbg 1,2,4,8 > gpurun_out/b_dbg.jsonl 2> gpurun_out/b_dbg.err || { tail -5 gpurun_out/b_dbg.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/b_dbg.jsonl'):
    d=json.loads(l); print(d['shape'],d['M'],'qmm',d['qmm_us'])
    for w in d['ws']: print('   ',{k:v for k,v in w.items() if k!='tflops'})
"
timeout -k 10 300 python -u tools/tune_qmm_ws.py --shapes qkv,wo,down --M 128,256 --cfgs 441412,242412,422212 > gpurun_out/b_ws2.jsonl 2> gpurun_out/b_ws2.err || { tail -5 gpurun_out/b_ws2.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/b_ws2.jsonl'):
    d=json.loads(l); b=d.get('best',{}); print(d['shape'],d['M'],'qmm',d['qmm_us'],'best',b.get('cfg'),b.get('splits'),b.get('us'),'x',d.get('speedup'),'err',max([w.get('rel_err',0) for w in d['ws']]))
"
