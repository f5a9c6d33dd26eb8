for bk in 2**20 2**21 2**22; do
  timeout -k 10 90 python3 -u scripts/dev/ktime.py --reps 4 --opt bucket_keys=$bk 2>&1 | grep total || exit 1
  timeout -k 10 90 python3 -u scripts/dev/ktime.py --reps 4 --dtype i64 --dist zipf --opt bucket_keys=$bk 2>&1 | grep total || exit 1
done
