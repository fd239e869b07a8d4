# rocprofv3 counter passes for the f16 qmm at the serving shapes (gate_up M=256): the best tuned tile vs
# a square-wave tile, to see whether MFMA, VALU, LDS or waiting bounds the kernel.
export PYTHONPATH=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT/gpurun_out
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT"
for c in "4,1,8,1,1" "2,2,4,33,1" "4,1,4,2,1"; do
  t=$(echo $c | tr , _)
  timeout -s KILL 90 rocprofv3 --pmc $P1 -d $R/pmcq_${t}_1 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/prof_qmm.py --shape gate_up --M 256 --cfg $c --iters 5 > $R/pmcq_${t}_1.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc $P2 -d $R/pmcq_${t}_2 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/prof_qmm.py --shape gate_up --M 256 --cfg $c --iters 5 > $R/pmcq_${t}_2.log 2>&1 || exit 1
  tail -1 $R/pmcq_${t}_1.log
done
cd $GRAFT_REPO_ROOT && python tools/pmc_summary.py gpurun_out/pmcq_* > gpurun_out/pmcq_summary.md 2>&1; tail -60 gpurun_out/pmcq_summary.md
