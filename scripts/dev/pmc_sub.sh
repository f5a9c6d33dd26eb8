#!/bin/bash
# PMC passes over one 2^30 sort (ktime.py, or SCRIPT): one rocprofv3 run per counter set, databases
# under gpurun_out/${TAG}pmc<i>.  ARGS = the script's arguments, TAG = output prefix.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
ARGS=${ARGS:-"--reps 1"}
SCRIPT=${SCRIPT:-scripts/dev/ktime.py}
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum" \
           "WRITE_SIZE" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d $R/gpurun_out/${TAG}pmc$i -o run -- python3 $R/$SCRIPT $ARGS > $R/gpurun_out/${TAG}pmc$i.log 2>&1 || exit $?
  echo "pmc pass $i ok"
done
