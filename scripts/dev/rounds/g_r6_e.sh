#!/bin/bash
# Round 6: the staged slow classify of the scatter (default build) and the batched one-key lookups
# of the histogram (build_variants/hb2, hb4) on mixed / few / uniform int32 and C4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
for d in mixed few uniform ref100; do
  VARS="hb2 hb4" ROUNDS=2 bash scripts/dev/ab_multi.sh --dist $d || exit $?
done
VARS="hb2 hb4" ROUNDS=2 bash scripts/dev/ab_multi.sh --dtype i64 --dist zipf || exit $?
