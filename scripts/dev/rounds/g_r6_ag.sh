set -o pipefail
mkdir -p gpurun_out
( VARS="t3 l3" ROUNDS=3 bash scripts/dev/ab_multi.sh --dtype i64 --dist uniform || exit $?
  VARS="t3 l3" ROUNDS=2 bash scripts/dev/ab_multi.sh --dtype i64 --dist zipf || exit $? ) > gpurun_out/r6_ab_nt_i64.log 2>&1
