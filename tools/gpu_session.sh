#!/bin/bash
# One gpurun session: GPU tests, then a short bench. Stops at the first crash/timeout.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD
TESTS=${TESTS:-tests}
timeout -k 10 ${TEST_TIMEOUT:-900} python -m pytest $TESTS -m gpu -q --timeout 240 -rf ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
if [ -n "${BENCH_ARGS+x}" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py $BENCH_ARGS > gpurun_out/bench.log 2>&1
  rc=$?
  echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
  exit $rc
fi
