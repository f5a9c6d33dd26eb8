#!/bin/bash
# Round-3 closing run: the fallback-rate probe of the B=2 sub-bucket case, then g_final.sh (GPU
# suite, stage timing, bench line, kernel-trace summaries).  Each GPU step has its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
REPS=20 timeout -k 10 240 python3 -u scripts/dev/dbg_k16.py > gpurun_out/fallback_rate.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/fallback_rate.log
bash scripts/dev/g_final.sh
