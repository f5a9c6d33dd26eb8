#!/bin/bash
# A/B of the default build against build_variants/<V> with ktime.py, alternating, plus a
# rocprofv3 kernel-trace summary of each.  usage: V=<variant> scripts/dev/ab_ktime.sh [ktime args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD; mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 90 python3 -u scripts/dev/ktime.py --reps 5 "$@" || exit $?
  DSORT_LIB=$R/build_variants/$V/libdsort.so timeout -k 10 90 python3 -u scripts/dev/ktime.py --reps 5 "$@" || exit $?
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/ab_def -o run -- python3 $R/scripts/dev/ktime.py --reps 5 "$@" > /dev/null 2>&1 || exit $?
DSORT_LIB=$R/build_variants/$V/libdsort.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/ab_var -o run -- python3 $R/scripts/dev/ktime.py --reps 5 "$@" > /dev/null 2>&1 || exit $?
for d in ab_def ab_var; do echo "== $d"; grep -h "bucket\|block_sort_w\|mergew\|sb_" $R/gpurun_out/$d/run_kernel_stats.csv | cut -d, -f1-4 | sed 's/(.*)//'; done
