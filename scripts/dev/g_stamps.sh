#!/bin/bash
# bucket/sort GPU tests, ktime A/B of $VS, and the line-scatter phase stamps of build_variants/stamps*
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_binsort.py tests/test_gpu_bucket.py tests/test_gpu_sort.py -q -x -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1
st=$?; echo "tests exit $st"; tail -2 gpurun_out/tests.log
[ $st -ne 0 ] && exit $st
VS="$VS" PREFIX=pv bash scripts/dev/g_pv.sh | grep -E "total|scatter_lines|==" || exit 1
for V in build_variants/stamps*; do echo "== $V"; DSORT_LIB=$PWD/$V/libdsort.so timeout -k 10 120 python3 scripts/dev/bkstamps.py || exit 1; done
