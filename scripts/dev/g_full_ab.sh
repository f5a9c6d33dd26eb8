#!/bin/bash
# Every GPU test, then bench A/B (default vs build_variants/$VS) at N=1: int32 metric and C4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -x -m gpu --timeout 170 --timeout-method thread > gpurun_out/tests.log 2>&1
st=$?; echo "tests exit $st"; tail -3 gpurun_out/tests.log
[ $st -ne 0 ] && exit $st
for r in 1 2; do
for V in default $VS; do
  L=""; [ "$V" != default ] && L="$PWD/build_variants/$V/libdsort.so"
  DSORT_LIB=$L timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$V.log 2>&1 || exit $?
  echo "$V i32 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_$V.log)"
  DSORT_LIB=$L timeout -k 10 200 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --dtype i64 --dist zipf > gpurun_out/bench64_$V.log 2>&1 || exit $?
  echo "$V i64zipf $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench64_$V.log)"
done
done
