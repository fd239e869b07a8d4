# qmm 256-row tiles (8,1,4,*) and 128x64 split-k wave tiles (4,2,4,2) vs the auto choice at serving M
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$PWD
L=gpurun_out/j17.log; : > $L
for sh in gate_up down qkv wo; do
  for M in 256 384; do
    timeout -k 10 60 python tools/prof_qmm.py --shape $sh --M $M --iters 20 >> $L 2>&1 || { tail -5 $L; exit 1; }
    for c in 8,1,4,1 8,1,4,2 4,2,4,2; do
      for sp in 1 2 4; do
        if [ $sp != 1 ] && { [ $sh = gate_up ] || [ $sh = qkv ]; }; then continue; fi
        timeout -k 10 60 python tools/prof_qmm.py --shape $sh --M $M --cfg $c,$sp --iters 20 >> $L 2>&1 || { tail -5 $L; exit 1; }
      done
    done
  done
done
grep -v amdgpu.ids $L
