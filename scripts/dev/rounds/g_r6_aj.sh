set -o pipefail
mkdir -p gpurun_out
( for d in sorted reverse few; do VARS="nont" ROUNDS=2 bash scripts/dev/ab_multi.sh --dtype i32 --dist $d || exit $?; done ) > gpurun_out/r6_ab_nt_other_inputs.log 2>&1
