# qmv A/B: current qmv.hip (weights issued before the activation prologue) vs the pre-e89a5a6 version,
# same box: decode GEMVs with the fused RMSNorm/q8 prologue at M=1 and the batch-1 engine bench
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$PWD
cp localai_tfp_amd/_lib/libmxk.so /tmp/libmxk_new.so
for v in new old new old; do
  if [ $v = old ]; then cp localai_tfp_amd/_lib_alt/libmxk.so localai_tfp_amd/_lib/libmxk.so; else cp /tmp/libmxk_new.so localai_tfp_amd/_lib/libmxk.so; fi
  for sh in gate_up down qkv wo; do
    timeout -k 10 60 python tools/prof_qmm.py --shape $sh --M 1 --gemv --iters 50 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" || exit 1
  done
done
for v in old new; do
  if [ $v = old ]; then cp localai_tfp_amd/_lib_alt/libmxk.so localai_tfp_amd/_lib/libmxk.so; else cp /tmp/libmxk_new.so localai_tfp_amd/_lib/libmxk.so; fi
  timeout -k 10 200 python bench.py --path engine --concurrency 1 --steps 100 --warmup 20 > gpurun_out/j21_$v.json 2> gpurun_out/j21_$v.err || { tail -5 gpurun_out/j21_$v.err; exit 1; }
  tail -1 gpurun_out/j21_$v.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$v' c1", d["value"], d["ms_per_step"])'
done
