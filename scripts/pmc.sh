#!/bin/bash
# PMC passes over scripts/kdriver.py (each pass its own run, no tracing domains besides kernels).
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-pmc}; shift
cd /tmp && export TMPDIR=/tmp
mkdir -p "$REPO/gpurun_out/$TAG"
i=0
for ctrs in "$@"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctrs -f csv -d "$REPO/gpurun_out/$TAG/p$i" -o run -- python3 "$REPO/scripts/kdriver.py" ${KARGS:---keys 2**28 --reps 1} > "$REPO/gpurun_out/$TAG/p$i.log" 2>&1 || { echo "pass $i ($ctrs) failed"; tail -3 "$REPO/gpurun_out/$TAG/p$i.log"; exit 1; }
  echo "pass $i ok: $ctrs"
done
