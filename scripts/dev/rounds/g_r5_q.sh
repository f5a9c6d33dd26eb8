#!/bin/bash
# Round 5: C4 (2^30 Zipf int64) back-to-back steps without stage events and stage times: default
# against build_variants/{noside,norb}, and the first level's oversampling at 64 / 128 (runtime option).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_sort.py tests/test_gpu_bucket.py > gpurun_out/r5q_tests.log 2>&1 || exit $?
sha256sum distributed-sorting-with-fault-tolerance_amd/lib/libdsort.so > gpurun_out/r5q_ab.log
for i in 1 2; do
  for V in noside norb; do
    echo "default: $(timeout -k 10 90 python3 scripts/dev/b2b.py --steps 10 --dtype i64 --dist zipf --timing 0 2>&1 | grep back-to-back)" >> gpurun_out/r5q_ab.log || exit $?
    echo "$V: $(DSORT_LIB=$R/build_variants/$V/libdsort.so timeout -k 10 90 python3 scripts/dev/b2b.py --steps 10 --dtype i64 --dist zipf --timing 0 2>&1 | grep back-to-back)" >> gpurun_out/r5q_ab.log || exit $?
  done
done
for o in 256 128 64; do
  timeout -k 10 90 python3 scripts/dev/ktime.py --reps 3 --dtype i64 --dist zipf --opt bucket_oversample=$o 2>&1 | grep -v amdgpu >> gpurun_out/r5q_ab.log || exit $?
done
timeout -k 10 90 python3 scripts/dev/ktime.py --reps 3 --dtype i64 2>&1 | grep -v amdgpu >> gpurun_out/r5q_ab.log || exit $?
timeout -k 10 90 python3 scripts/dev/ktime.py --reps 3 --dtype i64 --opt bucket_oversample=64 2>&1 | grep -v amdgpu >> gpurun_out/r5q_ab.log || exit $?
echo done
