#!/bin/bash
# Every GPU test, ktime of the three 2^30 configs, the N=1 bench line and a rocprofv3
# kernel-trace summary of the bench command.  Each GPU step has its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -x -m gpu --timeout 170 --timeout-method thread > gpurun_out/tests.log 2>&1
st=$?; echo "tests exit $st"; tail -3 gpurun_out/tests.log
[ $st -ne 0 ] && exit $st
timeout -k 10 120 python3 -u scripts/dev/ktime.py --reps 4 2>&1 | grep total || exit 1
timeout -k 10 120 python3 -u scripts/dev/ktime.py --reps 4 --dtype i64 --dist zipf 2>&1 | grep total || exit 1
timeout -k 10 120 python3 -u scripts/dev/ktime.py --reps 4 --dtype i64 2>&1 | grep total || exit 1
timeout -k 10 300 python3 -u bench.py > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
[ -n "$NO_PROF" ] && exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_bench -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_bench64 -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --dtype i64 --dist zipf > $R/gpurun_out/prof_bench64.log 2>&1 || exit $?
tail -1 $R/gpurun_out/prof_bench64.log
