#!/bin/bash
# rocprofv3 kernel-trace summary of the default bench workload (no PMC counters here).
# usage: scripts/profile.sh <tag> [bench args...]
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-prof}; shift
cd /tmp && export TMPDIR=/tmp
mkdir -p "$REPO/gpurun_out/$TAG"
timeout -k 10 ${PROF_TIMEOUT:-300} rocprofv3 --kernel-trace --stats -f csv -d "$REPO/gpurun_out/$TAG" -o run -- \
    python3 "$REPO/bench.py" --no-cpu-baseline "$@" > "$REPO/gpurun_out/$TAG/bench.log" 2>&1
st=$?
echo "profile exit $st"
find "$REPO/gpurun_out/$TAG" -name "*kernel_stats.csv" -exec cat {} \; | head -20
exit $st
