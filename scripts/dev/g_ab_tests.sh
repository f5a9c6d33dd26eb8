#!/bin/bash
# A/B of compile-time variants (ktime, 2 rounds) then the GPU suite against the variant $TESTV.
# usage: VS="v1 v2" TESTV=v2 scripts/dev/g_ab_tests.sh [ktime args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD; mkdir -p gpurun_out
bash scripts/dev/ab_multi.sh "$@" || exit $?
if [ -n "$TESTV" ]; then
  DSORT_LIB=$R/build_variants/$TESTV/libdsort.so timeout -k 10 400 python -u -m pytest tests -q -x -m gpu --timeout 170 --timeout-method thread > gpurun_out/tests_$TESTV.log 2>&1
  st=$?; echo "tests($TESTV) exit $st"; tail -3 gpurun_out/tests_$TESTV.log; exit $st
fi
