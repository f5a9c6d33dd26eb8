#!/bin/bash
# small:large tile targets of the skewed buckets (DSORT_BUCKET_SKEW), 2^30 int32, ktime.py
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for i in 1 2; do
  for v in ${SKEWS:-0 56:104 52:100 54:110 58:104 60:112}; do
    echo "== skew $v"
    DSORT_BUCKET_SKEW=$v timeout -k 10 90 python3 -u scripts/dev/ktime.py --reps 5 "$@" || exit $?
  done
done
