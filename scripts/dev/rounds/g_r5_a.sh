#!/bin/bash
# Round 5: stage timings of the adaptive int32 slot map, then the multi-rank / fault / plumbing GPU
# tests (host-transport status gates) and the adaptive-map parity tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for d in uniform byte ref100 few; do
  timeout -k 10 120 python3 -u scripts/dev/ktime.py --dist $d --reps 5 >> gpurun_out/r5a_ktime.log 2>&1 || exit $?
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_faults.py tests/test_gpu_ftsort.py \
    tests/test_gpu_plumbing.py "tests/test_gpu_sort.py::test_small_key_ranges_adaptive_map_bit_exact" \
    "tests/test_gpu_sort.py::test_small_key_ranges_other_sizes" -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/r5a_tests.log 2>&1
st=$?; tail -3 gpurun_out/r5a_tests.log; exit $st
