#!/bin/bash
# rocprofv3 kernel traces of scripts/dev/ktime.py for several library variants / env settings.
# usage: scripts/dev/prof_variants.sh "<tag>:<env assignments>" ...   (tag "x:DSORT_LIB=... K=V")
set -e
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd /tmp; export TMPDIR=/tmp; cd "$REPO"
for spec in "$@"; do
  tag=${spec%%:*}; envs=${spec#*:}
  P=${PREFIX:-pv}; mkdir -p "$REPO/gpurun_out/${P}_$tag"
  env $envs timeout -k 10 120 rocprofv3 --kernel-trace -d "$REPO/gpurun_out/${P}_$tag" -o run -- \
    python3 -u "$REPO/scripts/dev/ktime.py" --reps ${REPS:-3} $KTIME_ARGS > "$REPO/gpurun_out/${P}_$tag/ktime.log" 2>&1
  grep total "$REPO/gpurun_out/${P}_$tag/ktime.log" | grep -v SQLite
done
