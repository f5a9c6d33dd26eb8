#!/bin/bash
# Round-4 closing measurement on the GPU box, on the final build: the GPU suite, the PMC passes and
# kernel traces (scripts/dev/rounds/gpu_profile_r4.sh), a checked C3 rank, and the int32 / int64-Zipf bench
# lines.  Each GPU step has its own time limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/r4f_tests.log 2>&1
st=$?; tail -2 gpurun_out/r4f_tests.log; [ $st -ne 0 ] && exit $st
bash scripts/dev/rounds/gpu_profile_r4.sh pmc trace > gpurun_out/r4f_profile.log 2>&1 || exit $?
timeout -k 10 300 python3 -u scripts/c3_rank.py --steps 10 > gpurun_out/r4f_c3.json 2> gpurun_out/r4f_c3.err || exit $?
timeout -k 10 400 python3 -u bench.py > gpurun_out/r4f_bench_i32.json 2> gpurun_out/r4f_bench_i32.err || exit $?
timeout -k 10 300 python3 -u bench.py --dtype i64 --dist zipf --no-cpu-baseline > gpurun_out/r4f_bench_i64z.json 2> gpurun_out/r4f_bench_i64z.err || exit $?
echo final-done
