set -o pipefail
mkdir -p gpurun_out
( for i in 1 2; do
  for os in 128 64 96; do
    echo "== bucket_oversample=$os"
    timeout -k 10 90 python3 -u scripts/dev/ktime.py --reps 6 --dtype i64 --dist zipf --opt bucket_oversample=$os || exit $?
    timeout -k 10 90 python3 -u scripts/dev/ktime.py --reps 6 --dtype i32 --dist uniform --opt bucket_oversample=$os || exit $?
  done
done ) > gpurun_out/r6_ab_oversample_after_hash.log 2>&1
