#!/bin/bash
# A GPU test run on the current build: `scripts/gpu_tests.sh TAG [pytest args...]` (default: the
# whole suite, -m gpu), then smoke().  Output: gpurun_out/TAG_tests.log, TAG_smoke.log.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r6}; shift
mkdir -p gpurun_out
sha256sum distributed-sorting-with-fault-tolerance_amd/lib/libdsort.so > gpurun_out/${TAG}_tests.log
if [ $# -eq 0 ]; then set -- tests -m gpu; fi
timeout -k 10 1100 python -u -m pytest "$@" -x -v --timeout 250 --timeout-method thread >> gpurun_out/${TAG}_tests.log 2>&1
st=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $st -ne 0 ] && exit $st
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_smoke.log
