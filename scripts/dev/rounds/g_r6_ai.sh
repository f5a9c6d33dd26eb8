set -o pipefail
mkdir -p gpurun_out
( VARS="srev" ROUNDS=3 bash scripts/dev/ab_multi.sh --dtype i32 --dist uniform || exit $?
  VARS="srev" ROUNDS=2 bash scripts/dev/ab_multi.sh --dtype i64 --dist zipf || exit $? ) > gpurun_out/r6_ab_scatter_rev.log 2>&1
