#!/bin/bash
# Every GPU test, then ktime of the int32 metric sort and the int64 Zipf (C4) sort.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -x -m gpu --timeout 170 --timeout-method thread > gpurun_out/tests.log 2>&1
st=$?; echo "tests exit $st"; tail -4 gpurun_out/tests.log
[ $st -ne 0 ] && exit $st
timeout -k 10 120 python3 -u scripts/dev/ktime.py --reps 4 2>&1 | grep total || exit 1
timeout -k 10 120 python3 -u scripts/dev/ktime.py --reps 4 --dtype i64 --dist zipf 2>&1 | grep total || exit 1
timeout -k 10 120 python3 -u scripts/dev/ktime.py --reps 4 --dtype i64 2>&1 | grep total
