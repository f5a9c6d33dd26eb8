set -o pipefail
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sort.py tests/test_gpu_bucket.py -k "i64 or int64 or zipf" > gpurun_out/r6_hcb_tests.log 2>&1 || { tail -30 gpurun_out/r6_hcb_tests.log; exit 1; }
tail -3 gpurun_out/r6_hcb_tests.log
for d in zipf uniform; do VARS="hcb0 hcb2 hcb6" ROUNDS=2 bash scripts/dev/ab_multi.sh --dtype i64 --dist $d || exit $?; done > gpurun_out/r6_ab_hist_batch.log 2>&1
