# rocprofv3 counter passes for this round's kernel variants: qmm two-workgroups-per-CU tile (gate_up M=64)
# vs the one-workgroup tile, and the fused-input decode GEMV (gate_up, M=1). One pass per counter group.
export PYTHONPATH=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT/gpurun_out; P=$GRAFT_REPO_ROOT/tools/prof_qmm.py
SQ="SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
timeout -s KILL 90 rocprofv3 --pmc $SQ GRBM_GUI_ACTIVE -d $R/pmc_occ2 -o run --output-format csv -- python3 $P --shape gate_up --M 64 --cfg 2,1,4,18,1 --iters 5 > $R/pmc_occ2.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc $SQ GRBM_GUI_ACTIVE -d $R/pmc_occ1 -o run --output-format csv -- python3 $P --shape gate_up --M 64 --cfg 2,1,4,2,1 --iters 5 > $R/pmc_occ1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $R/pmc_occ2f -o run --output-format csv -- python3 $P --shape gate_up --M 64 --cfg 2,1,4,18,1 --iters 5 > $R/pmc_occ2f.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc $SQ GRBM_GUI_ACTIVE -d $R/pmc_gemv -o run --output-format csv -- python3 $P --shape gate_up --M 1 --gemv --iters 5 > $R/pmc_gemv.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $R/pmc_gemvf -o run --output-format csv -- python3 $P --shape gate_up --M 1 --gemv --iters 5 > $R/pmc_gemvf.log 2>&1
rc=$?
cd $GRAFT_REPO_ROOT
for n in occ2 occ1 gemv; do echo "== $n"; grep -E "us |TB/s" gpurun_out/pmc_$n.log | tail -1; done
python tools/pmc_summary.py gpurun_out/pmc_occ2 gpurun_out/pmc_occ2f > gpurun_out/pmc_occ2.md
python tools/pmc_summary.py gpurun_out/pmc_occ1 > gpurun_out/pmc_occ1.md
python tools/pmc_summary.py gpurun_out/pmc_gemv gpurun_out/pmc_gemvf > gpurun_out/pmc_gemv.md
cat gpurun_out/pmc_occ2.md gpurun_out/pmc_occ1.md gpurun_out/pmc_gemv.md | head -80
exit $rc
