#!/bin/bash
# Round-2 measurement set: PMC passes of the 2^30 int32 and int64-Zipf sorts, the rocprofv3
# kernel-trace summary of the bench command, and the bench lines.  Each GPU step has its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; mkdir -p gpurun_out
TAG=i32_ ARGS="--reps 1" bash scripts/dev/pmc_sub.sh || exit $?
TAG=i64_ ARGS="--reps 1 --dtype i64 --dist zipf" bash scripts/dev/pmc_sub.sh || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_bench -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_bench64 -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --dtype i64 --dist zipf > $R/gpurun_out/prof_bench64.log 2>&1 || exit $?
cd $R
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
timeout -k 10 300 python -u bench.py --dtype i64 --dist zipf --no-cpu-baseline > gpurun_out/bench64.log 2>&1 || exit $?
tail -1 gpurun_out/bench64.log
