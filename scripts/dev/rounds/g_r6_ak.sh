set -o pipefail
mkdir -p gpurun_out
( for d in sorted reverse uniform; do VARS="nont" ROUNDS=2 bash scripts/dev/ab_multi.sh --dtype i32 --dist $d || exit $?; done ) > gpurun_out/r6_ab_nt_ht.log 2>&1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_sort.py tests/test_gpu_bucket.py -k "sorted or hot or runs or reverse" > gpurun_out/r6_ht_tests.log 2>&1 || { tail -20 gpurun_out/r6_ht_tests.log; exit 1; }
tail -1 gpurun_out/r6_ht_tests.log
