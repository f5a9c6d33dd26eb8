#!/bin/bash
# int64 plan sweep: DSORT_BUCKETS x DSORT_MAX_LOGF on 2^30 keys (ktime.py stage times).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for dist in ${DISTS:-zipf uniform}; do
  for b in ${BUCKETS:-512 1024}; do
    for f in ${LOGFS:-4 5 6}; do
      echo "== dist=$dist B=$b logf=$f"
      DSORT_BUCKETS=$b DSORT_MAX_LOGF=$f timeout -k 10 90 python3 -u scripts/dev/ktime.py --dtype i64 --dist $dist --reps 3 || exit $?
    done
  done
done
