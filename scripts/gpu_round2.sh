#!/bin/bash
# Round-2 GPU check: every GPU test, then the N=1 bench, the 1-rank sample-sort path, and the
# refusal of --gpus 2 on a 1-GPU box.  Each GPU step has its own time limit; a crash/timeout ends it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest ${TESTS:-tests} -q -m gpu --timeout 170 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/tests.log 2>&1
st=$?
echo "tests exit $st"; tail -15 gpurun_out/tests.log
if [ $st -ne 0 ] && [ $st -ne 1 ]; then exit $st; fi
[ -n "$NO_BENCH" ] && exit $st
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 ${BENCH_ARGS} > gpurun_out/bench1.log 2>&1 || exit $?
tail -1 gpurun_out/bench1.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --path samplesort --no-cpu-baseline > gpurun_out/bench_ss1.log 2>&1 || exit $?
tail -1 gpurun_out/bench_ss1.log
timeout -k 10 120 python -u bench.py --gpus 2 --steps 2 > gpurun_out/bench_g2.log 2>&1
echo "bench --gpus 2 exit $? (2 expected)"; tail -2 gpurun_out/bench_g2.log
exit $st
