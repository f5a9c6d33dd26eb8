set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bucket.py tests/test_gpu_faults.py tests/test_gpu_multirank.py -k "16k or c3 or large or multirank or oversized or bucket_exchange" > gpurun_out/r6_big_tests.log 2>&1 || { tail -30 gpurun_out/r6_big_tests.log; exit 1; }
tail -3 gpurun_out/r6_big_tests.log
for i in 1 2; do
  timeout -k 10 120 python3 -u scripts/c3_rank.py --steps 5 --warmup 2 --only-bx || exit $?
  DSORT_LIB=$PWD/build_variants/big0/libdsort.so timeout -k 10 120 python3 -u scripts/c3_rank.py --steps 5 --warmup 2 --only-bx || exit $?
done > gpurun_out/r6_ab_c3_bigchunk.log 2>&1
