set -o pipefail
mkdir -p gpurun_out
( VARS="fillnt" ROUNDS=3 bash scripts/dev/ab_multi.sh --dtype i64 --dist zipf || exit $?
  VARS="fillnt" ROUNDS=2 bash scripts/dev/ab_multi.sh --dtype i32 --dist few || exit $? ) > gpurun_out/r6_ab_fill_nt.log 2>&1
