#!/bin/bash
# Round 5: A/B of the scatter's batched classify / unguarded loads and the histogram's batched lookup
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
VARS="cb0 cb0g0 cb2 cb8 h4 h8" bash scripts/dev/ab_multi.sh > gpurun_out/r5b_ab.log 2>&1 || exit $?
for d in byte ref100 few sorted; do
  timeout -k 10 120 python3 -u scripts/dev/ktime.py --dist $d --reps 5 2>&1 | grep -v amdgpu.ids >> gpurun_out/r5b_ab.log || exit $?
done
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > gpurun_out/r5b_bench.json 2> gpurun_out/r5b_bench.err || exit $?
echo done
