#!/bin/bash
# Round 4: one rank of config C3 on one MI355X (scripts/c3_rank.py): the local sort of 2^29 int32
# keys and the F = 8 receive merge of 8 x 2^26, then their rocprofv3 kernel trace and PMC traffic.
#   scripts/g_r4_c3.sh [TAG]   outputs gpurun_out/${TAG}c3_*
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; mkdir -p gpurun_out
TAG=${1:-r4_}
timeout -k 10 200 python3 -u scripts/c3_rank.py --steps 10 > gpurun_out/${TAG}c3_rank.json 2> gpurun_out/${TAG}c3_rank.err || exit $?
cat gpurun_out/${TAG}c3_rank.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/${TAG}c3_trace -o run -- python3 $R/scripts/c3_rank.py --steps 5 --no-check > $R/gpurun_out/${TAG}c3_trace.log 2>&1 || exit $?
if [ -n "$PMC" ]; then
  i=0
  for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
             "WRITE_SIZE" "FETCH_SIZE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $set -d $R/gpurun_out/${TAG}c3_pmc$i -o run -- python3 $R/scripts/c3_rank.py --steps 1 --warmup 0 --no-check > $R/gpurun_out/${TAG}c3_pmc$i.log 2>&1 || exit $?
    echo "pmc pass $i ok"
  done
fi
echo c3-done
