#!/bin/bash
# skewed bucket sizes (default) vs equal buckets (DSORT_BUCKET_SKEW=0), 2^30 int32, ktime.py
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for i in 1 2 3; do
  echo "== skew"; unset DSORT_BUCKET_SKEW
  timeout -k 10 90 python3 -u scripts/dev/ktime.py --reps 5 "$@" || exit $?
  echo "== equal"; export DSORT_BUCKET_SKEW=0
  timeout -k 10 90 python3 -u scripts/dev/ktime.py --reps 5 "$@" || exit $?
done
