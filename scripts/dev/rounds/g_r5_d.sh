#!/bin/bash
# Round 5: the round-4 library and the guarded-load variant against the current build, int64 Zipf
# and int32 uniform, one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
VARS="r4 g0" bash scripts/dev/ab_multi.sh --dtype i64 --dist zipf > gpurun_out/r5d_ab.log 2>&1 || exit $?
VARS="r4 g0" bash scripts/dev/ab_multi.sh >> gpurun_out/r5d_ab.log 2>&1 || exit $?
VARS="r4" bash scripts/dev/ab_multi.sh --dtype i64 >> gpurun_out/r5d_ab.log 2>&1 || exit $?
echo done
