set -o pipefail
mkdir -p gpurun_out
( VARS="idsnt" ROUNDS=3 bash scripts/dev/ab_multi.sh --dtype i64 --dist zipf || exit $? ) > gpurun_out/r6_ab_ids_nt.log 2>&1
