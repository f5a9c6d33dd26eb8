#!/bin/bash
# GPU-box smoke: parity tests then a short bench.  Stops at the first crash/timeout
# (exit status other than 0 = pass, 1 = test failure).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TESTS=${TESTS:-tests/test_gpu_sort.py}
timeout -k 10 ${TEST_TIMEOUT:-400} python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/tests.log 2>&1
st=$?
echo "tests exit $st"; tail -5 gpurun_out/tests.log
if [ $st -ne 0 ] && [ $st -ne 1 ]; then exit $st; fi
if [ -n "$BENCH_ARGS" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-300} python -u bench.py $BENCH_ARGS > gpurun_out/bench.log 2>&1
  bst=$?
  echo "bench exit $bst"; tail -3 gpurun_out/bench.log
  exit $bst
fi
exit $st
