set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 200 python -u tools/dbg/rwkv_gpu2.py > gpurun_out/a_rwkv.log 2>&1; echo "rwkv rc=$?"; grep -v amdgpu.ids gpurun_out/a_rwkv.log | tail -8
timeout -k 10 300 python -u tools/tune_qmm_ws.py --shapes gate_up,qkv,wo,down --M 128,256 --cfgs 22211,41411,12111 > gpurun_out/a_ws.jsonl 2> gpurun_out/a_ws.err || { tail -20 gpurun_out/a_ws.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/a_ws.jsonl'):
    d=json.loads(l); b=d.get('best',{}); print(d['shape'],d['M'],'qmm',d['qmm_us'],'best',b.get('cfg'),b.get('splits'),b.get('us'),'x',d.get('speedup'),'errs',max([w.get('rel_err',0) for w in d['ws']]))
"
export PYTHONPATH=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT/gpurun_out
for arm in "ws 41411,1" "cfg 4,1,4,2,1"; do
  set -- $arm; t=$(echo $1_$2 | tr , _)
  timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE -d $R/pmcw_${t} -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/prof_qmm.py --shape gate_up --M 128 --$1 $2 --iters 5 > $R/pmcw_${t}.log 2>&1 || exit 1
  tail -1 $R/pmcw_${t}.log
done
cd $GRAFT_REPO_ROOT && python tools/pmc_summary.py gpurun_out/pmcw_* > gpurun_out/pmcw_summary.md 2>&1; grep -A8 "qmm" gpurun_out/pmcw_summary.md | head -40
