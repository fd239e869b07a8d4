set -o pipefail
R=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 120 python -u tools/dbg/graph_launch_mb.py 350 > $R/gmb_default.json && \
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 120 python -u tools/dbg/graph_launch_mb.py 350 > $R/gmb_pc0.json && \
DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 timeout -k 10 120 python -u tools/dbg/graph_launch_mb.py 350 > $R/gmb_pc1.json
