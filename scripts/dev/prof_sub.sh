#!/bin/bash
# Per-kernel stats of the 2^30 sorts (int32 uniform, int64 Zipf) + the correctness sweep.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/ps32 -o run -- python3 $R/scripts/dev/ktime.py --reps 3 > $R/gpurun_out/ps32.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/ps64 -o run -- python3 $R/scripts/dev/ktime.py --dtype i64 --dist zipf --reps 3 > $R/gpurun_out/ps64.log 2>&1 || exit $?
cd $R && timeout -k 10 400 python -u scripts/dev/subcheck.py > gpurun_out/subcheck.log 2>&1
