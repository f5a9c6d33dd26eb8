#!/bin/bash
# Round 5: phase stamps (DSORT_STAMPS build) of the bin sort, the first-level scatter and the local
# partition at 2^30 int32 on the current kernels.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export DSORT_LIB=$PWD/build_variants/stamps/libdsort.so
for s in binstamps.py "bkstamps.py i32" "bkstamps.py i64z" sbstamps.py; do
  echo "== $s" >> gpurun_out/r5_stamps.log
  timeout -k 10 120 python3 -u scripts/dev/$s 2>&1 | grep -v amdgpu.ids >> gpurun_out/r5_stamps.log || exit $?
done
echo done
