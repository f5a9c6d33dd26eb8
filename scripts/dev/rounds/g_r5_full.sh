#!/bin/bash
# Round 5: the whole GPU suite (pytest -m gpu) on the current build, then smoke().
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
sha256sum distributed-sorting-with-fault-tolerance_amd/lib/libdsort.so > gpurun_out/r5_full_tests.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread >> gpurun_out/r5_full_tests.log 2>&1
st=$?; tail -3 gpurun_out/r5_full_tests.log; [ $st -ne 0 ] && exit $st
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5_smoke.log 2>&1 || exit $?
cat gpurun_out/r5_smoke.log | tail -1
