#!/bin/bash
# Round-6 measurement set on the final build: the library's sha256 as run on the box, PMC passes
# (separate runs, scripts/dev/pmc_sub.sh) of the 2^30 int32 and int64-Zipf sorts, the rocprofv3
# kernel-trace summaries of both bench commands, and the C3 rank.  Every GPU step has its own time
# limit; the script stops at the first failure.   scripts/gpu_profile_r6.sh [pmc] [trace] [c3]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; mkdir -p gpurun_out
sha256sum distributed-sorting-with-fault-tolerance_amd/lib/libdsort.so > gpurun_out/pmc_lib_sha256.txt
WHAT=${*:-pmc trace c3}
if [[ " $WHAT " == *" pmc "* ]]; then
  TAG=r6i32_ ARGS="--reps 1" bash scripts/dev/pmc_sub.sh || exit $?
  TAG=r6i64_ ARGS="--reps 1 --dtype i64 --dist zipf" bash scripts/dev/pmc_sub.sh || exit $?
fi
cd /tmp && export TMPDIR=/tmp
if [[ " $WHAT " == *" trace "* ]]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/r6prof_bench -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/r6prof_bench.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/r6prof_bench64 -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --dtype i64 --dist zipf > $R/gpurun_out/r6prof_bench64.log 2>&1 || exit $?
fi
if [[ " $WHAT " == *" c3 "* ]]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/r6prof_c3 -o run -- python3 $R/scripts/c3_rank.py --steps 3 --warmup 1 --no-check --only-bx > $R/gpurun_out/r6prof_c3.log 2>&1 || exit $?
fi
echo profile-done
