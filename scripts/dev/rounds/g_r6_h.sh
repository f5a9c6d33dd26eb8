#!/bin/bash
# Round 6: first-level oversampling 128 (default) against 64 / 96 (build_variants), bench-like
# back-to-back steps, int32 uniform and C4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
R=$PWD
for i in 1 2 3; do
  for v in "" os64 os96; do
    if [ -n "$v" ]; then export DSORT_LIB=$R/build_variants/$v/libdsort.so; else unset DSORT_LIB; fi
    echo -n "${v:-default} i32: "; timeout -k 10 60 python3 -u scripts/dev/b2b.py --steps 20 --timing 0 2>&1 | grep back || exit 1
  done
done
for v in "" os64; do
  if [ -n "$v" ]; then export DSORT_LIB=$R/build_variants/$v/libdsort.so; else unset DSORT_LIB; fi
  echo -n "${v:-default} C4: "; timeout -k 10 60 python3 -u scripts/dev/b2b.py --steps 10 --timing 0 --dtype i64 --dist zipf 2>&1 | grep back || exit 1
done
