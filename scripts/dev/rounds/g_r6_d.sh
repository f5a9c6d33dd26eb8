#!/bin/bash
# Round 6: phase stamps of the first-level scatter on [1,100]-mixed-with-uniform and 16-distinct-key
# input against uniform (DSORT_STAMPS build).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export DSORT_LIB=$PWD/build_variants/stamps/libdsort.so
for s in i32 mixed few; do
  echo "== bkstamps $s"
  timeout -k 10 120 python3 -u scripts/dev/bkstamps.py $s 2>&1 | grep -v amdgpu.ids || exit $?
done
