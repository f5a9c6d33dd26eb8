#!/bin/bash
# Round 5: GPU bucket/sort tests on the current build, then stage times of the default build against
# build_variants/$V at 2^30 Zipf int64 (C4), uniform int32, 16 distinct int32 keys, uniform int64
# (or the ';'-separated ktime.py argument sets of $ARGS_LIST).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_sort.py tests/test_gpu_bucket.py > gpurun_out/${TAG}_tests.log 2>&1 || exit $?
sha256sum distributed-sorting-with-fault-tolerance_amd/lib/libdsort.so > gpurun_out/${TAG}_ab.log
IFS=";" read -ra LIST <<< "${ARGS_LIST:---dtype i64 --dist zipf;--dtype i32;--dtype i32 --dist few;--dtype i64}"
for a in "${LIST[@]}"; do
  for i in 1 2; do
    timeout -k 10 90 python3 scripts/dev/ktime.py --reps 3 $a 2>&1 | grep -v amdgpu >> gpurun_out/${TAG}_ab.log || exit $?
    DSORT_LIB=$R/build_variants/$V/libdsort.so timeout -k 10 90 python3 scripts/dev/ktime.py --reps 3 $a 2>&1 | grep -v amdgpu >> gpurun_out/${TAG}_ab.log || exit $?
  done
done
echo done
