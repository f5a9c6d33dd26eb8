set -o pipefail
mkdir -p gpurun_out
( VARS="s12g2 s15g2" ROUNDS=3 bash scripts/dev/ab_multi.sh --dtype i32 --dist uniform || exit $? ) > gpurun_out/r6_ab_local32_pairs.log 2>&1
