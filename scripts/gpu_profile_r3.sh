#!/bin/bash
# Round-3 measurement set: PMC passes (separate runs, scripts/dev/pmc_sub.sh) of the 2^30 int32 and
# int64-Zipf sorts, and the rocprofv3 kernel-trace summaries of the bench command.  Every GPU step
# has its own time limit; the script stops at the first failure.
#   scripts/gpu_profile_r3.sh [pmc] [trace]     (default: both)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; mkdir -p gpurun_out
WHAT=${*:-pmc trace}
if [[ " $WHAT " == *" pmc "* ]]; then
  TAG=r3i32_ ARGS="--reps 1" bash scripts/dev/pmc_sub.sh || exit $?
  TAG=r3i64_ ARGS="--reps 1 --dtype i64 --dist zipf" bash scripts/dev/pmc_sub.sh || exit $?
fi
if [[ " $WHAT " == *" trace "* ]]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/r3prof_bench -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/r3prof_bench.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/r3prof_bench64 -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --dtype i64 --dist zipf > $R/gpurun_out/r3prof_bench64.log 2>&1 || exit $?
fi
echo profile-done
