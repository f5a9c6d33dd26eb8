#!/bin/bash
# Round 4 iteration on the GPU box: selected GPU tests (TESTS, pytest -k expression or file list),
# then the C3 rank measurement (scripts/c3_rank.py), then a short bench line.  Each GPU step has its
# own time limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r4_}
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -q --timeout 250 --timeout-method thread > gpurun_out/${TAG}tests.log 2>&1
  st=$?; tail -3 gpurun_out/${TAG}tests.log; [ $st -ne 0 ] && exit $st
fi
if [ -n "$C3" ]; then
  timeout -k 10 300 python3 -u scripts/c3_rank.py --steps 10 > gpurun_out/${TAG}c3_rank.json 2> gpurun_out/${TAG}c3_rank.err || exit $?
  cat gpurun_out/${TAG}c3_rank.json
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline $BENCH > gpurun_out/${TAG}bench.json 2> gpurun_out/${TAG}bench.err || exit $?
  cat gpurun_out/${TAG}bench.json
fi
echo iter-done
