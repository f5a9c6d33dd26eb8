set -o pipefail
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sort.py tests/test_gpu_bucket.py tests/test_gpu_multirank.py -k "i64 or int64 or zipf or multirank" > gpurun_out/r6_ohash_tests.log 2>&1 || { tail -30 gpurun_out/r6_ohash_tests.log; exit 1; }
tail -3 gpurun_out/r6_ohash_tests.log
for d in zipf uniform; do VARS="ohash0" ROUNDS=2 bash scripts/dev/ab_multi.sh --dtype i64 --dist $d || exit $?; done > gpurun_out/r6_ab_onekey_hash.log 2>&1
