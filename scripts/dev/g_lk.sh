#!/bin/bash
# bucket/sort GPU tests for the default build and build_variants in $TV, then ktime A/B of $VS.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for V in default $TV; do
  L=""; [ "$V" != default ] && L="$PWD/build_variants/$V/libdsort.so"
  DSORT_LIB=$L timeout -k 10 400 python -u -m pytest tests/test_gpu_binsort.py tests/test_gpu_bucket.py tests/test_gpu_sort.py -q -x -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests_$V.log 2>&1
  st=$?; echo "tests $V exit $st"; tail -1 gpurun_out/tests_$V.log
  [ $st -ne 0 ] && exit $st
done
VS="$VS" PREFIX=pv bash scripts/dev/g_pv.sh | grep -E "total|scatter_lines|sb_local|bin_sort_kernel<int|==" || exit 1
