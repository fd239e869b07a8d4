#!/bin/bash
# The one documented profiling entry point (run on the GPU box through gpurun; writes under gpurun_out/,
# copy the summaries you want to keep into profiles/):
#
#   bash tools/gpu_profile.sh engine [CONC] [STEPS]   rocprofv3 kernel trace of the in-process engine bench at
#                                                    concurrency CONC (default 128): per-kernel table per step
#   bash tools/gpu_profile.sh window [CONC] [STEPS] [WIN_MS]  the same from a rocpd trace, restricted to the last WIN_MS
#                                                    of kernels: per-step tables (decode-only / mixed) and launch gaps
#   bash tools/gpu_profile.sh pmc SHAPE M CFG          counter passes (MFMA / VALU / LDS / waits) of one qmm2
#                                                    configuration "wm,ks,wn,splits" on a Llama-3-8B projection
#   bash tools/gpu_profile.sh gemm [MS] [SHAPES]       default (untuned-rule) GEMM dispatch against M, one-launch vs
#                                                    256-row chunks (JSONL; the tuned plans: MX_TUNE_REPORT)
#
# Every GPU step runs under its own timeout; counter passes stay within the per-block slot limits (8 SQ).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$R"
export PYTHONUNBUFFERED=1 PYTHONPATH=${GRAFT_REPO_ROOT:-$(pwd)}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mode=$1; shift
case "$mode" in
  engine)
    conc=${1:-128}; steps=${2:-40}
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/prof_engine_c$conc" -o run --output-format csv -- \
      python3 "$ROOT/bench.py" --path engine --concurrency "$conc" --steps "$steps" --warmup 5 --step-group 1 --min-ttft-samples 0 ${MODEL:+--model $MODEL} ${BENCH_ARGS} > "$R/prof_engine_c$conc.log" 2>&1 || exit 1
    cd "$ROOT" && python tools/prof_summary.py "$R/prof_engine_c$conc" --top 40 --steps "$steps" > "$R/prof_engine_c$conc.md"
    tail -45 "$R/prof_engine_c$conc.md"
    ;;
  window)
    # rocpd trace of the engine bench; table over the last WIN ms (the steady state, after tuning / capture), per-step
    # split (decode-only vs mixed) by the step's first kernel (the embedding gather) and the inter-kernel gaps
    conc=${1:-128}; steps=${2:-200}; win=${3:-1000}
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 600 rocprofv3 --kernel-trace -d "$R/profw_c$conc" -o run -- \
      python3 "$ROOT/bench.py" --path engine --concurrency "$conc" --steps "$steps" --warmup 5 --step-group 1 --min-ttft-samples 0 ${MODEL:+--model $MODEL} ${BENCH_ARGS} > "$R/profw_c$conc.log" 2>&1 || exit 1
    db=$(find "$R/profw_c$conc" -name '*.db' | head -1)
    cd "$ROOT" && python tools/rocpd_summary.py "$db" --window-ms "$win" --split-steps dequant_rows --gaps --top 30 > "$R/profw_c$conc.md" || exit 1
    rm -rf "$R/profw_c$conc"
    head -40 "$R/profw_c$conc.md"
    ;;
  pmc)
    shape=$1; M=$2; cfg=$3; t=$(echo "$cfg" | tr , _)
    P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU"
    P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT"
    cd /tmp && export TMPDIR=/tmp
    for p in 1 2; do
      eval PP=\$P$p
      timeout -s KILL 90 rocprofv3 --pmc $PP -d "$R/pmc_${shape}_${M}_${t}_$p" -o run --output-format csv -- \
        python3 "$ROOT/tools/prof_qmm.py" --shape "$shape" --M "$M" --q2 "$cfg" --iters 5 > "$R/pmc_${shape}_${M}_${t}_$p.log" 2>&1 || exit 1
    done
    cd "$ROOT" && python tools/pmc_summary.py "$R"/pmc_${shape}_${M}_${t}_* > "$R/pmc_${shape}_${M}_${t}.md"
    cat "$R/pmc_${shape}_${M}_${t}.md"
    ;;
  gemm)
    MS=${1:-128,192,256,320,384,512} SHAPES=${2:-gate_up,qkv,wo,down,down_q6} \
      timeout -k 10 600 python -u tools/gemm_curve.py > "$R/gemm_curve.jsonl" || exit 1
    cat "$R/gemm_curve.jsonl"
    ;;
  *)
    sed -n 2,12p "$0"; exit 2 ;;
esac
