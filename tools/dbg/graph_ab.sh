set -o pipefail
R=$GRAFT_REPO_ROOT/gpurun_out
B="python -u bench.py --path engine --steps 60 --warmup 10"
timeout -k 10 300 $B --no-graphs > $R/ab_nographs.json 2>/dev/null && \
DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 timeout -k 10 300 $B > $R/ab_pc1.json 2>/dev/null && \
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 300 $B > $R/ab_pc0.json 2>/dev/null && \
timeout -k 10 300 $B > $R/ab_default.json 2>/dev/null
