#!/bin/bash
# Round 6 closing measurement of the current build: the GPU suite + smoke, the PMC passes (int32
# uniform, int64 Zipf, the C3 rank) and the PMC table keyed to this build, the kernel-trace
# summaries of the bench commands, then the bench lines (int32 with the CPU baseline; C4; the text
# codec with its kernel trace; the one-GPU sample sort with its C3/C4/C5 legs) and the
# input-dependent timings.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
R=$PWD; mkdir -p gpurun_out
T=${TAG:-r6}
if [ -z "$NOTEST" ]; then bash scripts/gpu_tests.sh ${T}_full || exit $?; fi
bash scripts/gpu_profile_r6.sh pmc trace c3 > gpurun_out/${T}_profile.log 2>&1 || exit $?
TAG=r6c3_ SCRIPT=scripts/c3_rank.py ARGS="--steps 1 --warmup 1 --no-check --only-bx" bash scripts/dev/pmc_sub.sh >> gpurun_out/${T}_profile.log 2>&1 || exit $?
python3 scripts/dev/pmc_json.py gpurun_out/r6_pmc_traffic.json r6i32_ r6i64_ > gpurun_out/${T}_pmc_json.log 2>&1 || exit $?
cp gpurun_out/r6_pmc_traffic.json profiles/r6_pmc_traffic.json || exit $?
timeout -k 10 600 python3 bench.py > gpurun_out/${T}_bench_i32.json 2> gpurun_out/${T}_bench_i32.err || exit $?
timeout -k 10 300 python3 bench.py --no-cpu-baseline --dtype i64 --dist zipf > gpurun_out/${T}_bench_i64zipf.json 2> gpurun_out/${T}_bench_i64zipf.err || exit $?
timeout -k 10 400 python3 bench.py --gpus 1 --path samplesort --no-cpu-baseline > gpurun_out/${T}_bench_ss_legs.json 2> gpurun_out/${T}_bench_ss_legs.err || exit $?
for d in uniform mixed few ref100 sorted reverse; do
  timeout -k 10 120 python3 -u scripts/dev/ktime.py --reps 6 --dist $d >> gpurun_out/${T}_input_timings.log 2>&1 || exit $?
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/${T}prof_codec -o run -- python3 $R/bench.py --codec --keys 2**28 --steps 5 --warmup 2 > $R/gpurun_out/${T}_bench_codec.json 2> $R/gpurun_out/${T}_bench_codec.err || exit $?
echo final-done
