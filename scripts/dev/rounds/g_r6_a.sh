#!/bin/bash
# Round 6: the wave-fence self-test, the 1-GPU samplesort bench with its C3/C4/C5 legs, and a
# kernel-trace timeline of back-to-back 2^30 int32 sorts (idle gaps).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
R=$PWD; mkdir -p gpurun_out
timeout -k 10 600 python3 -u bench.py --gpus 1 --path samplesort --steps 5 --warmup 2 --no-cpu-baseline \
  > gpurun_out/r6b_bench_ss_legs.json 2> gpurun_out/r6b_bench_ss_legs.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace -f csv -d $R/gpurun_out/r6_tl -o run -- python3 $R/scripts/dev/b2b.py --steps 4 --timing 0 > $R/gpurun_out/r6_tl.log 2>&1 || exit $?
python3 $R/scripts/dev/timeline.py $R/gpurun_out/r6_tl/run_kernel_trace.csv >> $R/gpurun_out/r6_tl.log 2>&1
echo done-a
