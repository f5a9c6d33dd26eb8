set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_sort.py tests/test_gpu_bucket.py tests/test_gpu_multirank.py > gpurun_out/r6_blk_tests.log 2>&1 || { tail -30 gpurun_out/r6_blk_tests.log; exit 1; }
tail -2 gpurun_out/r6_blk_tests.log
( VARS="blk0" ROUNDS=3 bash scripts/dev/ab_multi.sh --dtype i32 --dist uniform || exit $?
  VARS="blk0" ROUNDS=2 bash scripts/dev/ab_multi.sh --dtype i64 --dist zipf || exit $? ) > gpurun_out/r6_ab_gather_blk.log 2>&1
