# A/B of the dense (hipBLASLt f16 weight cache) vs quantised-MFMA routing thresholds on the engine bench.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
run() {
  env "$@" timeout -k 10 200 python bench.py --path engine --steps 200 --warmup 150 > gpurun_out/exp.log 2>&1 || exit $?
  echo "$* $(grep '^{' gpurun_out/exp.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["host_ms_per_step"]["fwd"])')"
}
run MX_DENSE_MIN_M_SWIGLU=96
run MX_DENSE_MIN_M_SWIGLU=512
run MX_DENSE_MIN_M_SWIGLU=512 MX_DENSE_MIN_M_NOSPLIT=512
run MX_DENSE_MIN_M_SWIGLU=96
