#!/bin/bash
# Round 6: the refined slot (BkMap.r2s) -- its parity tests, then the input-dependent timings again.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
bash scripts/gpu_tests.sh r6c tests/test_gpu_sort.py tests/test_gpu_multirank.py tests/test_gpu_bucket.py \
  -k "adaptive or small_key or bit_exact or onekey or one_key or few or narrow or extremes" || exit $?
for d in uniform mixed few ref100; do
  timeout -k 10 120 python3 -u scripts/dev/ktime.py --reps 6 --dist $d || exit $?
done
