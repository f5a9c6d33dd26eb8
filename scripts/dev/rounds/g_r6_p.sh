set -o pipefail
mkdir -p gpurun_out
( for i in 1 2; do
    timeout -k 10 120 python3 -u scripts/c3_rank.py --steps 5 --warmup 2 --only-bx --no-check | grep '^{' || exit $?
    DSORT_LIB=$PWD/build_variants/pscan64/libdsort.so timeout -k 10 120 python3 -u scripts/c3_rank.py --steps 5 --warmup 2 --only-bx --no-check | grep '^{' || exit $?
  done ) > gpurun_out/r6_ab_pieces_scan64.log 2>&1
