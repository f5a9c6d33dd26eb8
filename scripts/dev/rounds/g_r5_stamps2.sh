#!/bin/bash
# Round 5: bin sort phase stamps (DSORT_STAMPS build) at 2^30 int32 and at 2^30 Zipf int64 (C4).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export DSORT_LIB=$PWD/build_variants/stamps/libdsort.so
for s in "binstamps.py i64z" binstamps.py; do
  echo "== $s" >> gpurun_out/r5_stamps2.log
  timeout -k 10 120 python3 -u scripts/dev/$s 2>&1 | grep -v amdgpu.ids >> gpurun_out/r5_stamps2.log || exit $?
done
echo done
