#!/bin/bash
# Round 5 (session 2): stage times and a kernel trace of back-to-back 2^30 int32 sorts (timeline of
# one step with its idle gaps), on the build as committed.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; mkdir -p gpurun_out
sha256sum distributed-sorting-with-fault-tolerance_amd/lib/libdsort.so > gpurun_out/r5f_ktime.log
timeout -k 10 120 python3 -u scripts/dev/ktime.py --reps 5 2>&1 | grep -v amdgpu.ids >> gpurun_out/r5f_ktime.log || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $R/gpurun_out/r5f_b2b -o run -- python3 $R/scripts/dev/b2b.py --steps 6 > $R/gpurun_out/r5f_b2b.log 2>&1 || exit $?
cd $R
python3 scripts/dev/timeline.py $(ls gpurun_out/r5f_b2b/*/run_kernel_trace.csv gpurun_out/r5f_b2b/run_kernel_trace.csv 2>/dev/null | head -1) > gpurun_out/r5f_timeline.txt
echo done
