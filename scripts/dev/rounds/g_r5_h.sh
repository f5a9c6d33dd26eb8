#!/bin/bash
# Round 5: GPU sort/bucket tests on the current build, then back-to-back bench-style steps
# (scripts/dev/b2b.py: host gaps included) and device stage times of the default build against
# build_variants/$VARS, interleaved.    VARS="v1 v2" TAG=x [B2B="--timing 0"] [NOTEST=1] scripts/dev/rounds/g_r5_h.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; mkdir -p gpurun_out
if [ -z "$NOTEST" ]; then
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_sort.py tests/test_gpu_bucket.py > gpurun_out/${TAG}_tests.log 2>&1 || exit $?
fi
sha256sum distributed-sorting-with-fault-tolerance_amd/lib/libdsort.so > gpurun_out/${TAG}_ab.log
for i in 1 2 3; do
  for V in $VARS; do
    echo "default: $(timeout -k 10 90 python3 scripts/dev/b2b.py --steps 20 $B2B 2>&1 | grep back-to-back)" >> gpurun_out/${TAG}_ab.log || exit $?
    echo "$V: $(DSORT_LIB=$R/build_variants/$V/libdsort.so timeout -k 10 90 python3 scripts/dev/b2b.py --steps 20 $B2B 2>&1 | grep back-to-back)" >> gpurun_out/${TAG}_ab.log || exit $?
  done
done
for V in $VARS; do
  timeout -k 10 90 python3 -u scripts/dev/ktime.py --reps 5 2>&1 | grep -v amdgpu.ids >> gpurun_out/${TAG}_ab.log || exit $?
  DSORT_LIB=$R/build_variants/$V/libdsort.so timeout -k 10 90 python3 -u scripts/dev/ktime.py --reps 5 2>&1 | grep -v amdgpu.ids >> gpurun_out/${TAG}_ab.log || exit $?
done
echo done
