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
  [ $rc -ne 0 ] && exit $rc
fi
if [ -n "${PROF_ARGS+x}" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 ${PROF_TIMEOUT:-600} rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" $PROF_ARGS > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1
  rc=$?
  cd "$GRAFT_REPO_ROOT"
  echo "prof rc=$rc"; tail -3 gpurun_out/prof.log
  find gpurun_out/prof -name "*stats*" | head
  exit $rc
fi
