#!/bin/bash
# Kernel trace of a few back-to-back 2^30 sorts (ktime.py) for scripts/dev/timeline.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $R/gpurun_out/ktrace -o run -- python3 $R/scripts/dev/ktime.py --reps 3 "$@" > $R/gpurun_out/ktrace.log 2>&1 || exit $?
grep total $R/gpurun_out/ktrace.log
