#!/bin/bash
# Round 5: GPU text codec tests, then bench.py --codec (2^28 keys) for the default build and each of
# build_variants/$VARS, interleaved twice.    VARS="v1 v2" TAG=x scripts/dev/rounds/g_r5_cod.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_text.py > gpurun_out/${TAG}_tests.log 2>&1 || exit $?
sha256sum distributed-sorting-with-fault-tolerance_amd/lib/libdsort.so > gpurun_out/${TAG}_ab.log
for i in 1 2; do
  for V in default $VARS; do
    L=""; [ "$V" != default ] && L=$R/build_variants/$V/libdsort.so
    echo "$V: $(DSORT_LIB=$L timeout -k 10 120 python3 bench.py --codec --keys 2**28 --steps 5 --warmup 2 --no-cpu-baseline 2>&1 | grep metric | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("format_ms", d["format_ms"], "parse_ms", d["parse_ms"])')" >> gpurun_out/${TAG}_ab.log || exit $?
  done
done
echo done
