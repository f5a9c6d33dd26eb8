set -o pipefail
mkdir -p gpurun_out
( VARS="ntboth" ROUNDS=4 bash scripts/dev/ab_multi.sh --dtype i32 --dist uniform || exit $?
  VARS="ntboth" ROUNDS=3 bash scripts/dev/ab_multi.sh --dtype i64 --dist zipf || exit $? ) > gpurun_out/r6_ab_nt_both.log 2>&1
