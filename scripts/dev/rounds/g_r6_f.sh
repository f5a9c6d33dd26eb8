#!/bin/bash
# Round 6: the scatter's prefetch behind the classify (default) against in front of it
# (build_variants/early), interleaved, on uniform / mixed / few int32 and C4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
for d in uniform mixed few; do
  VARS="early" ROUNDS=3 bash scripts/dev/ab_multi.sh --dist $d || exit $?
done
VARS="early" ROUNDS=2 bash scripts/dev/ab_multi.sh --dtype i64 --dist zipf || exit $?
