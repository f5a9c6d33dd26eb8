set -o pipefail
mkdir -p gpurun_out
( VARS="sntl gntl" ROUNDS=3 bash scripts/dev/ab_multi.sh --dtype i32 --dist uniform || exit $?
  VARS="sntl gntl" ROUNDS=2 bash scripts/dev/ab_multi.sh --dtype i64 --dist zipf || exit $? ) > gpurun_out/r6_ab_nt_loads.log 2>&1
