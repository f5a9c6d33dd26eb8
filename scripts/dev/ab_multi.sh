#!/bin/bash
# ktime.py of the default build and of every build_variants/<V> in turn (2 rounds).
# usage: VS="v1 v2" scripts/dev/ab_multi.sh [ktime args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD; mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 90 python3 -u scripts/dev/ktime.py --reps 4 "$@" || exit $?
  for V in $VS; do
    DSORT_LIB=$R/build_variants/$V/libdsort.so timeout -k 10 90 python3 -u scripts/dev/ktime.py --reps 4 "$@" || exit $?
  done
done
