#!/bin/bash
# Round-4 measurement set: PMC passes (separate runs, scripts/dev/pmc_sub.sh) of the 2^30 int32 and
# int64-Zipf sorts, the rocprofv3 kernel-trace summaries of the bench command, and the C3 rank
# (scripts/c3_rank.py) trace.  Every GPU step has its own time limit; the script stops at the first
# failure.   scripts/dev/rounds/gpu_profile_r4.sh [pmc] [trace] [c3]     (default: all)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; mkdir -p gpurun_out
WHAT=${*:-pmc trace c3}
if [[ " $WHAT " == *" pmc "* ]]; then
  TAG=r4i32_ ARGS="--reps 1" bash scripts/dev/pmc_sub.sh || exit $?
  TAG=r4i64_ ARGS="--reps 1 --dtype i64 --dist zipf" bash scripts/dev/pmc_sub.sh || exit $?
fi
cd /tmp && export TMPDIR=/tmp
if [[ " $WHAT " == *" trace "* ]]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/r4prof_bench -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/r4prof_bench.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/r4prof_bench64 -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --dtype i64 --dist zipf > $R/gpurun_out/r4prof_bench64.log 2>&1 || exit $?
fi
if [[ " $WHAT " == *" c3 "* ]]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/r4prof_c3 -o run -- python3 $R/scripts/c3_rank.py --steps 3 --warmup 1 --no-check > $R/gpurun_out/r4prof_c3.log 2>&1 || exit $?
fi
echo profile-done
