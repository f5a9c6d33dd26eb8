#!/bin/bash
# GPU tests (stop at first failure), then rocprof kernel traces of ktime for the default build
# and build_variants listed in $VS ($KTIME_ARGS passed through).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 ${TEST_TIMEOUT:-400} python -u -m pytest ${TESTS:-tests} -q -x -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1
st=$?; echo "tests exit $st"; tail -${TAILN:-4} gpurun_out/tests.log
[ $st -ne 0 ] && exit $st
VS="$VS" bash scripts/dev/g_pv.sh
