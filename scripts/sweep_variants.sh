#!/bin/bash
# A/B of compile-time variants: VARIANTS="minw4 minw6" scripts/sweep_variants.sh [bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for V in $VARIANTS; do
  DSORT_LIB=$PWD/build_variants/$V/libdsort.so timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps ${STEPS:-5} --warmup 2 "$@" > gpurun_out/var_$V.log 2>&1 || { echo "variant $V failed"; tail -5 gpurun_out/var_$V.log; exit 1; }
  python - "$V" <<'PY'
import json,sys
V=sys.argv[1]
d=json.loads(open(f"gpurun_out/var_{V}.log").read().strip().splitlines()[-1])
print(f"{V}: value={d['value']/1e9:.2f} Gkeys/s ms={d['ms_per_step']:.2f} merge_kernel_ms={d['roofline']['avg_pass_ms']} block_ms={d['roofline']['block_sort_ms']}")
PY
done
