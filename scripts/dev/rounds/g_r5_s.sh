#!/bin/bash
# Round 5: first-level oversampling 256 vs 128 samples per bucket, back-to-back steps without stage
# events (the nested splitter sort is inside the step; ktime.py's device total starts after it).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2 3; do
  for o in 256 128; do
    echo "i32 os=$o: $(timeout -k 10 90 python3 scripts/dev/b2b.py --steps 20 --timing 0 --opt bucket_oversample=$o 2>&1 | grep back-to-back)" >> gpurun_out/r5s_os.log || exit $?
    echo "i64z os=$o: $(timeout -k 10 90 python3 scripts/dev/b2b.py --steps 10 --timing 0 --dtype i64 --dist zipf --opt bucket_oversample=$o 2>&1 | grep back-to-back)" >> gpurun_out/r5s_os.log || exit $?
  done
done
echo done
