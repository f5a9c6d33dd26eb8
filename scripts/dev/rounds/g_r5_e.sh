#!/bin/bash
# Round 5: stage times of the current build (int32 uniform, int64 Zipf), a kernel trace of
# back-to-back sorts (one step's idle gaps: scripts/dev/timeline.py), the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; mkdir -p gpurun_out
sha256sum distributed-sorting-with-fault-tolerance_amd/lib/libdsort.so > gpurun_out/r5e_ktime.log
for a in "" "--dtype i64 --dist zipf"; do
  timeout -k 10 120 python3 -u scripts/dev/ktime.py --reps 5 $a 2>&1 | grep -v amdgpu.ids >> gpurun_out/r5e_ktime.log || exit $?
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $R/gpurun_out/r5e_b2b -o run -- python3 $R/scripts/dev/b2b.py --steps 6 > $R/gpurun_out/r5e_b2b.log 2>&1 || exit $?
cd $R
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > gpurun_out/r5e_bench.json 2> gpurun_out/r5e_bench.err || exit $?
echo done
