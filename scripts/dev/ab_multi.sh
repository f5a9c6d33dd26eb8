#!/bin/bash
# Interleaved A/B of the default build and build_variants/$VARS with ktime.py (stage device times of
# the fastest of --reps sorts), ROUNDS times.   VARS="v1 v2" [ROUNDS=3] scripts/dev/ab_multi.sh [ktime args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
for i in $(seq ${ROUNDS:-3}); do
  timeout -k 10 90 python3 -u scripts/dev/ktime.py --reps 6 "$@" || exit $?
  for v in $VARS; do
    DSORT_LIB=$R/build_variants/$v/libdsort.so timeout -k 10 90 python3 -u scripts/dev/ktime.py --reps 6 "$@" || exit $?
  done
done
