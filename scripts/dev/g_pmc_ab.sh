#!/bin/bash
# SQ counter passes (2 sets) of ktime for the default build and build_variants in $VS.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
ARGS=${ARGS:-"--reps 1"}
for V in default $VS; do
  L=""; [ "$V" != default ] && L="DSORT_LIB=$R/build_variants/$V/libdsort.so"
  i=0
  for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_BRANCH"; do
    i=$((i+1))
    env $L X=1 timeout -s KILL 90 rocprofv3 --pmc $set -d $R/gpurun_out/pmc_${V}_$i -o run -- python3 $R/scripts/dev/ktime.py $ARGS > $R/gpurun_out/pmc_${V}_$i.log 2>&1 || exit $?
  done
done
cd $R && python3 scripts/dev/pmc_ab_summary.py ${FILTER:-bin_sort} | tee gpurun_out/pmc_ab.txt
