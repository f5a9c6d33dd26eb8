set -o pipefail
mkdir -p gpurun_out
export DSORT_LIB=$PWD/build_variants/ohash3/libdsort.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sort.py tests/test_gpu_bucket.py tests/test_gpu_multirank.py > gpurun_out/r6_ohash3_tests.log 2>&1 || { tail -30 gpurun_out/r6_ohash3_tests.log; exit 1; }
tail -3 gpurun_out/r6_ohash3_tests.log
unset DSORT_LIB
for d in few mixed ref100 uniform; do VARS="ohash3" ROUNDS=2 bash scripts/dev/ab_multi.sh --dtype i32 --dist $d || exit $?; done > gpurun_out/r6_ab_onekey_hash_i32.log 2>&1
