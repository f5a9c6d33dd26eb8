#!/bin/bash
# A/B of the default build against several build_variants/<V> with ktime.py in one GPU session,
# interleaved (default, V1, default, V2, ...) twice.  usage: VARS="v1 v2" scripts/dev/ab_multi.sh [ktime args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD; mkdir -p gpurun_out
sha256sum distributed-sorting-with-fault-tolerance_amd/lib/libdsort.so
for i in 1 2; do
  for V in $VARS; do
    timeout -k 10 90 python3 -u scripts/dev/ktime.py --reps 5 "$@" 2>&1 | grep -v amdgpu.ids || exit $?
    DSORT_LIB=$R/build_variants/$V/libdsort.so timeout -k 10 90 python3 -u scripts/dev/ktime.py --reps 5 "$@" 2>&1 | grep -v amdgpu.ids || exit $?
  done
done
