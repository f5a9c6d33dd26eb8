#!/bin/bash
# rocprof kernel traces of ktime for the default build and build_variants listed in $VS
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD; mkdir -p gpurun_out
specs="default:X=1"
for V in $VS; do specs="$specs $V:DSORT_LIB=$R/build_variants/$V/libdsort.so"; done
bash scripts/dev/prof_variants.sh $specs || exit $?
python3 scripts/dev/pv_summary.py > gpurun_out/${PREFIX:-pv}_summary.txt
cat gpurun_out/${PREFIX:-pv}_summary.txt
