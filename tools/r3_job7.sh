# qmm on Q4_K vs MX4F (pre-decoded f16 sub-block scale/offset) at the serving shapes and tiles: is the per-tile
# Q4_K scale decode a bottleneck?
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$PWD
for sh in gate_up qkv down; do
  for M in 128 256 2048; do
    for qt in 12 3; do
      timeout -k 10 60 python tools/prof_qmm.py --shape $sh --M $M --qt $qt --iters 20 >> gpurun_out/j7_cmp.log 2>&1 || { tail -5 gpurun_out/j7_cmp.log; exit 1; }
    done
  done
done
grep -v amdgpu.ids gpurun_out/j7_cmp.log
