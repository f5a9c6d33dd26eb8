set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bucket.py tests/test_gpu_faults.py tests/test_gpu_multirank.py -k "c3 or tile_cap or tile_table or large or oversized or bucket_exchange or pure" > gpurun_out/r6_pe_tests.log 2>&1 || { tail -30 gpurun_out/r6_pe_tests.log; exit 1; }
tail -2 gpurun_out/r6_pe_tests.log
( for i in 1 2 3; do
    timeout -k 10 120 python3 -u scripts/c3_rank.py --steps 5 --warmup 2 --only-bx --no-check | grep '^{' || exit $?
    DSORT_LIB=$PWD/build_variants/pe0/libdsort.so timeout -k 10 120 python3 -u scripts/c3_rank.py --steps 5 --warmup 2 --only-bx --no-check | grep '^{' || exit $?
  done ) > gpurun_out/r6_ab_pieces_early.log 2>&1
