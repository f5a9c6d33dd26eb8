#!/bin/bash
# per-bucket fan-in vs the global plan at 768 / 1024 buckets (2^30 int32, ktime.py).  The bucket
# count is set through the nominal bucket size: DSORT_BUCKETS would also bucket the int64 sort of
# the splitter samples.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for i in 1 2; do
  for b in ${BS:-768 1024}; do
    for m in per global; do
      echo "== B=$b fanin=$m"
      if [ $m = global ]; then export DSORT_BUCKET_FANIN=global; else unset DSORT_BUCKET_FANIN; fi
      DSORT_BUCKET_KEYS=$((1073741824 / b)) timeout -k 10 90 python3 -u scripts/dev/ktime.py --reps 5 "$@" || exit $?
    done
  done
done
