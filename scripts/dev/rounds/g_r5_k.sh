#!/bin/bash
# Round 5: the int32 histogram with the packed, batched lookups (default) against the unpacked one
# (build_variants/nohp): GPU bucket/sort tests, stage times for uniform, few, [1, 100], sorted keys.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_sort.py tests/test_gpu_bucket.py > gpurun_out/r5k_tests.log 2>&1 || exit $?
VARS="nohp" bash scripts/dev/ab_multi.sh > gpurun_out/r5k_ab.log 2>&1 || exit $?
for d in few ref100 sorted byte; do
  timeout -k 10 90 python3 scripts/dev/ktime.py --reps 3 --dist $d 2>&1 | grep -v amdgpu >> gpurun_out/r5k_ab.log || exit $?
  DSORT_LIB=$R/build_variants/nohp/libdsort.so timeout -k 10 90 python3 scripts/dev/ktime.py --reps 3 --dist $d 2>&1 | grep -v amdgpu >> gpurun_out/r5k_ab.log || exit $?
done
echo done
