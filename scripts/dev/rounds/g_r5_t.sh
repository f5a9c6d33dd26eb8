#!/bin/bash
# Round 5: second-level scan variants.  GPU sort/bucket tests on the current build, then kernel-trace
# summaries of ktime.py (2^30 int32 and C4) and of the C3 rank for the default build and each of
# build_variants/$VARS (TAG names the outputs).      VARS="v1 v2" TAG=x scripts/dev/rounds/g_r5_t.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; mkdir -p gpurun_out
if [ -z "$NOTEST" ]; then
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_sort.py tests/test_gpu_bucket.py tests/test_gpu_multirank.py > gpurun_out/${TAG}_tests.log 2>&1 || exit $?
fi
sha256sum distributed-sorting-with-fault-tolerance_amd/lib/libdsort.so > gpurun_out/${TAG}_ab.log
for V in default $VARS; do
  L=""; [ "$V" != default ] && L=$R/build_variants/$V/libdsort.so
  for a in "--dtype i32" "--dtype i64 --dist zipf"; do
    n=$(echo "$a" | tr -d ' -')
    DSORT_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/${TAG}_${V}_$n -o run -- python3 $R/scripts/dev/ktime.py --reps 3 $a >> gpurun_out/${TAG}_ab.log 2>&1 || exit $?
  done
  DSORT_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/${TAG}_${V}_c3 -o run -- python3 $R/scripts/c3_rank.py --steps 3 --warmup 1 --only-bx >> gpurun_out/${TAG}_ab.log 2>&1 || exit $?
done
if [ -n "$STAMPS" ]; then
  for d in i32 i64; do DSORT_LIB=$R/build_variants/$STAMPS/libdsort.so timeout -k 10 120 python3 scripts/dev/scanstamps.py $d 2>&1 | grep -v amdgpu >> gpurun_out/${TAG}_ab.log || exit $?; done
fi
echo done
