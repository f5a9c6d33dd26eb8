#!/bin/bash
# Round 6: input-dependent timings at 2^30 int32 (uniform, 16 distinct keys, [1,100], [1,100] mixed
# half and half with uniform keys, sorted, reversed) and the C3 rank through the bench's leg.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
for d in uniform few ref100 mixed sorted reverse; do
  timeout -k 10 120 python3 -u scripts/dev/ktime.py --reps 6 --dist $d || exit $?
done
timeout -k 10 300 python3 -u bench.py --gpus 1 --path samplesort --steps 5 --warmup 2 --no-cpu-baseline --legs c3 \
  > gpurun_out/r6_c3leg.json 2> gpurun_out/r6_c3leg.err || exit $?
grep '^{' gpurun_out/r6_c3leg.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); l=d['legs']['c3']; print('c3 leg', l['keys'], l['ms_per_step'], l['verified'], l['roofline']['kernel'], l['roofline']['frac'])"
