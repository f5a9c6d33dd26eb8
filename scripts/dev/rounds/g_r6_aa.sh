set -o pipefail
mkdir -p gpurun_out
( VARS="idsall" ROUNDS=3 bash scripts/dev/ab_multi.sh --dtype i64 --dist uniform || exit $? ) > gpurun_out/r6_ab_ids_all_i64.log 2>&1
