#!/bin/bash
# Round 5: A/B of the scatter's batched placement and pipelined line phase (int32 and int64 Zipf),
# then the bucket / sort GPU tests on the default build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
VARS="p0lu1 p0 lu1 p8 lu4 bb32 bb32g4 sg3 sg5" bash scripts/dev/ab_multi.sh > gpurun_out/r5c_ab.log 2>&1 || exit $?
VARS="p0lu1" bash scripts/dev/ab_multi.sh --dtype i64 --dist zipf >> gpurun_out/r5c_ab.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_bucket.py tests/test_gpu_sort.py -x -q --timeout 200 \
    --timeout-method thread > gpurun_out/r5c_tests.log 2>&1
st=$?; tail -3 gpurun_out/r5c_tests.log; exit $st
