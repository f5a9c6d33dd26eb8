set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_sort.py tests/test_gpu_bucket.py > gpurun_out/r6_vpc_tests.log 2>&1 || { tail -30 gpurun_out/r6_vpc_tests.log; exit 1; }
tail -2 gpurun_out/r6_vpc_tests.log
( for d in uniform; do VARS="vpc0" ROUNDS=2 bash scripts/dev/ab_multi.sh --dtype i32 --dist $d || exit $?; done
  VARS="vpc0" ROUNDS=2 bash scripts/dev/ab_multi.sh --dtype i64 --dist zipf || exit $?
  for i in 1 2; do
    timeout -k 10 120 python3 -u scripts/c3_rank.py --steps 5 --warmup 2 --only-bx --no-check | grep '^{' || exit $?
    DSORT_LIB=$PWD/build_variants/vpc0/libdsort.so timeout -k 10 120 python3 -u scripts/c3_rank.py --steps 5 --warmup 2 --only-bx --no-check | grep '^{' || exit $?
  done ) > gpurun_out/r6_ab_gather_vpc.log 2>&1
