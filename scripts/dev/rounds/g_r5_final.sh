#!/bin/bash
# Round 5 closing measurement of the current build: the GPU suite + smoke, the PMC passes (int32
# uniform, int64 Zipf, the C3 rank), the kernel-trace summaries of the bench commands and the C3
# rank, then the bench lines (int32 with the CPU baseline; C4; the text codec with its kernel trace).  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; mkdir -p gpurun_out
bash scripts/dev/rounds/g_r5_full.sh || exit $?
bash scripts/dev/rounds/gpu_profile_r5.sh pmc trace c3 > gpurun_out/r5_profile.log 2>&1 || exit $?
TAG=r5c3_ SCRIPT=scripts/c3_rank.py ARGS="--steps 1 --warmup 1 --no-check --only-bx" bash scripts/dev/pmc_sub.sh >> gpurun_out/r5_profile.log 2>&1 || exit $?
# the PMC table of this build, made on the box so the bench lines below find it matched
python3 scripts/dev/pmc_json.py gpurun_out/r5_pmc_traffic.json r5i32_ r5i64_ > gpurun_out/r5_pmc_json.log 2>&1 || exit $?
cp gpurun_out/r5_pmc_traffic.json profiles/r5_pmc_traffic.json || exit $?
timeout -k 10 600 python3 bench.py > gpurun_out/r5_bench_i32.json 2> gpurun_out/r5_bench_i32.err || exit $?
timeout -k 10 300 python3 bench.py --no-cpu-baseline --dtype i64 --dist zipf > gpurun_out/r5_bench_i64zipf.json 2> gpurun_out/r5_bench_i64zipf.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/r5prof_codec -o run -- python3 $R/bench.py --codec --keys 2**28 --steps 5 --warmup 2 > $R/gpurun_out/r5_bench_codec.json 2> $R/gpurun_out/r5_bench_codec.err || exit $?
echo final-done
