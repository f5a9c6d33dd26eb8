set -o pipefail
mkdir -p gpurun_out
( VARS="l64g1" ROUNDS=3 bash scripts/dev/ab_multi.sh --dtype i64 --dist zipf || exit $?
  VARS="l64g1" ROUNDS=2 bash scripts/dev/ab_multi.sh --dtype i64 --dist uniform || exit $? ) > gpurun_out/r6_ab_local64_g1.log 2>&1
