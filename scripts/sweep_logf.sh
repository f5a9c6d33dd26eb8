#!/bin/bash
# A/B of the k-way fan-in cap (DSORT_MAX_LOGF) on the default bench workload.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for L in ${LOGFS:-3 4 5 6}; do
  DSORT_MAX_LOGF=$L timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps ${STEPS:-5} --warmup 2 $EXTRA > gpurun_out/sweep_$L.log 2>&1 || { echo "logf $L failed"; tail -5 gpurun_out/sweep_$L.log; exit 1; }
  python - "$L" <<'PY'
import json,sys
L=sys.argv[1]
d=json.loads(open(f"gpurun_out/sweep_{L}.log").read().strip().splitlines()[-1])
print(f"logf={L} value={d['value']/1e9:.2f} Gkeys/s ms={d['ms_per_step']:.2f} merge_kernel_ms={d['roofline']['avg_pass_ms']} frac={d['roofline']['frac']} block_ms={d['roofline']['block_sort_ms']} cfg={d['config']['workload']}")
PY
done
