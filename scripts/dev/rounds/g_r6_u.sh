set -o pipefail
mkdir -p gpurun_out
( VARS="l64g2 l64g3" ROUNDS=2 bash scripts/dev/ab_multi.sh --dtype i64 --dist zipf || exit $?
  VARS="l64g2 l64g3" ROUNDS=2 bash scripts/dev/ab_multi.sh --dtype i64 --dist uniform || exit $? ) > gpurun_out/r6_ab_local64.log 2>&1
