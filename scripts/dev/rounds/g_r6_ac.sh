set -o pipefail
mkdir -p gpurun_out
( VARS="linesnt idsnt" ROUNDS=2 bash scripts/dev/ab_multi.sh --dtype i32 --dist uniform || exit $?
  VARS="linesnt idsnt" ROUNDS=2 bash scripts/dev/ab_multi.sh --dtype i64 --dist zipf || exit $? ) > gpurun_out/r6_ab_lines_nt.log 2>&1
