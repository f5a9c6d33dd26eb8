#!/bin/bash
# GPU tests ($TESTS), then per-kernel times of the default build and build_variants in $VS for the
# int32 metric sort and the int64 Zipf sort (C4).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 ${TEST_TIMEOUT:-400} python -u -m pytest ${TESTS:-tests} -q -x -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1
st=$?; echo "tests exit $st"; tail -3 gpurun_out/tests.log
[ $st -ne 0 ] && exit $st
VS="$VS" PREFIX=pv bash scripts/dev/g_pv.sh || exit $?
VS="$VS" PREFIX=pv64 KTIME_ARGS="--dtype i64 --dist zipf" bash scripts/dev/g_pv.sh
