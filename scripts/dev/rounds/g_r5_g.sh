#!/bin/bash
# Round 5: A/B of compile-time variants (scripts/dev/ab_multi.sh) and kernel traces of back-to-back
# sorts for the default build and one variant (one step's timeline: scripts/dev/timeline.py).
#   VARS="v1 v2" TRACEVAR=v1 TAG=x scripts/dev/rounds/g_r5_g.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; mkdir -p gpurun_out
bash scripts/dev/ab_multi.sh > gpurun_out/${TAG}_ab.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $R/gpurun_out/${TAG}_b2b -o run -- python3 $R/scripts/dev/b2b.py --steps 6 > $R/gpurun_out/${TAG}_b2b.log 2>&1 || exit $?
if [ -n "$TRACEVAR" ]; then
  DSORT_LIB=$R/build_variants/$TRACEVAR/libdsort.so timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $R/gpurun_out/${TAG}_b2b_var -o run -- python3 $R/scripts/dev/b2b.py --steps 6 > $R/gpurun_out/${TAG}_b2b_var.log 2>&1 || exit $?
fi
echo done
