for d in 0 1 2; do for c in "128 4,1,4,1" "256 4,1,8,1" "2048 4,2,8,1"; do set -- $c; MX_QMM_DBG=$d timeout -k 5 60 python tools/prof_qmm.py --shape gate_up --M $1 --cfg $2 --iters 20 | sed "s/^/dbg=$d /"; done; done
for d in 0 1 2; do MX_QMM_DBG=$d timeout -k 5 60 python tools/prof_qmm.py --shape down --M 256 --cfg 4,1,4,4 --iters 20 | sed "s/^/dbg=$d /"; done
