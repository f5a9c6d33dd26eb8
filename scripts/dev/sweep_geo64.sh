#!/bin/bash
# int64 tile geometry variants (scripts/build_variant.sh builds) on 2^30 keys, ktime.py stage times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for v in ${VARIANTS:-default k16 t1024}; do
  for dist in zipf uniform; do
    if [ $v = default ]; then unset DSORT_LIB; else export DSORT_LIB=$PWD/build_variants/$v/libdsort.so; fi
    for f in ${LOGFS:-4 5}; do
      echo "== $v dist=$dist logf=$f"
      DSORT_MAX_LOGF=$f timeout -k 10 90 python3 -u scripts/dev/ktime.py --dtype i64 --dist $dist --reps 3 || exit $?
    done
  done
done
