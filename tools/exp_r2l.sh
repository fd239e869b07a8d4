# qmm WN=2 / two-column-group tiles (each LDS A fragment feeds two MFMAs) at M = 96..256: correctness of
# every config vs the dense fp32 product (inside the sweep) and timings vs the current choice / dense.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 600 env SHAPES=gate_up,down,qkv MS=96,128,192,256 python -u tools/tune_qmm.py > gpurun_out/l_tune.jsonl 2> gpurun_out/l_tune.err || { tail gpurun_out/l_tune.err; exit 1; }
python tools/sum_tune.py gpurun_out/l_tune.jsonl
