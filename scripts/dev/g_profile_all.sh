#!/bin/bash
# The measurement set of the current build in one call: PMC passes of the 2^30 int32 and int64-Zipf
# sorts -> profiles/r3_pmc_traffic.json (copied to gpurun_out/, which is what comes back), then
# scripts/dev/g_final.sh (GPU suite, stage timing, the bench line -- its `traffic` read from that
# JSON -- and the kernel-trace summaries).  Each GPU step has its own limit; stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD; mkdir -p gpurun_out
bash scripts/gpu_profile_r3.sh pmc > gpurun_out/profile_pmc.log 2>&1 || { tail -5 gpurun_out/profile_pmc.log; exit 1; }
cd "$R"
python3 scripts/dev/pmc_json.py profiles/r3_pmc_traffic.json r3i32_ r3i64_ || exit 1
cp profiles/r3_pmc_traffic.json gpurun_out/r3_pmc_traffic.json
bash scripts/dev/g_final.sh
