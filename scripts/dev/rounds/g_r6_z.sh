set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_sort.py tests/test_gpu_bucket.py -k "i64 or int64 or zipf" > gpurun_out/r6_hrb_tests.log 2>&1 || { tail -30 gpurun_out/r6_hrb_tests.log; exit 1; }
tail -2 gpurun_out/r6_hrb_tests.log
( VARS="hrb0" ROUNDS=3 bash scripts/dev/ab_multi.sh --dtype i64 --dist zipf || exit $?
  VARS="hrb0" ROUNDS=2 bash scripts/dev/ab_multi.sh --dtype i64 --dist uniform || exit $? ) > gpurun_out/r6_ab_hist_rb.log 2>&1
