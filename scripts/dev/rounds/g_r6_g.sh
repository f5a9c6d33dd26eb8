#!/bin/bash
# Round 6: A/B of the current build against build_variants/prev (back-to-back steps, bench-like),
# plus a kernel-trace timeline of the current build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
R=$PWD
for i in 1 2 3; do
  timeout -k 10 60 python3 -u scripts/dev/b2b.py --steps 20 --timing 0 || exit $?
  DSORT_LIB=$R/build_variants/prev/libdsort.so timeout -k 10 60 python3 -u scripts/dev/b2b.py --steps 20 --timing 0 || exit $?
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace -f csv -d $R/gpurun_out/r6_tl2 -o run -- python3 $R/scripts/dev/b2b.py --steps 4 --timing 0 > /dev/null 2>&1 || exit $?
python3 $R/scripts/dev/timeline.py $R/gpurun_out/r6_tl2/run_kernel_trace.csv bucket_sample_kernel
