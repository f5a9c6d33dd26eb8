#!/bin/bash
# int64 per-bucket fan-in vs the global plan, 512 / 1024 buckets, 2^30 Zipf and uniform (ktime.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for dist in zipf uniform; do
  for b in ${BS:-512 1024}; do
    for m in per global; do
      echo "== $dist B=$b fanin=$m"
      if [ $m = global ]; then export DSORT_BUCKET_FANIN=global; else unset DSORT_BUCKET_FANIN; fi
      DSORT_BUCKETS=$b timeout -k 10 90 python3 -u scripts/dev/ktime.py --dtype i64 --dist $dist --reps 3 || exit $?
    done
  done
done
