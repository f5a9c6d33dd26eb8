#!/bin/bash
# One iteration on the GPU box: the whole GPU suite, ktime of the three 2^30 configs, then
# optional phase stamps of a DSORT_STAMPS variant (STAMPS=<variant>).  Each step has its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -x -m gpu --timeout 170 --timeout-method thread > gpurun_out/tests.log 2>&1
st=$?; echo "tests exit $st"; tail -3 gpurun_out/tests.log
[ $st -ne 0 ] && exit $st
timeout -k 10 120 python3 -u scripts/dev/ktime.py --reps 4 2>&1 | grep total || exit 1
timeout -k 10 120 python3 -u scripts/dev/ktime.py --reps 4 --dtype i64 --dist zipf 2>&1 | grep total || exit 1
timeout -k 10 120 python3 -u scripts/dev/ktime.py --reps 4 --dtype i64 2>&1 | grep total || exit 1
if [ -n "$STAMPS" ]; then
  DSORT_LIB=$R/build_variants/$STAMPS/libdsort.so timeout -k 10 120 python3 -u scripts/dev/bkstamps.py 2>&1 | grep -v amdgpu.ids || exit 1
  DSORT_LIB=$R/build_variants/$STAMPS/libdsort.so timeout -k 10 120 python3 -u scripts/dev/binstamps.py 2>&1 | grep -v amdgpu.ids || exit 1
fi
