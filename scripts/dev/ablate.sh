#!/bin/bash
# Times compile-time ablation variants built by scripts/build_variant.sh (no verification):
#   VARIANTS="a b" bash scripts/dev/ablate.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
timeout -k 5 120 python3 scripts/dev/ktime.py || exit 1
for V in $VARIANTS; do
  DSORT_LIB=$PWD/build_variants/$V/libdsort.so timeout -k 5 120 python3 scripts/dev/ktime.py || { echo "variant $V failed"; exit 1; }
done
