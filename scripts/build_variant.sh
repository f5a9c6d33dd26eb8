#!/bin/bash
# Build libdsort with extra compile flags into build_variants/<name>/libdsort.so
# usage: scripts/build_variant.sh <name> "<hipcc flags>"
set -e
REPO="$(cd "$(dirname "$0")/.." && pwd)"
PKG="$REPO/distributed-sorting-with-fault-tolerance_amd"
OUT="$REPO/build_variants/$1"; mkdir -p "$OUT/obj"
for f in dsort_wave dsort_text dsort_api; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I"$REPO/include" -I"$PKG/csrc" -munsafe-fp-atomics $2 \
    -c "$PKG/csrc/$f.hip" -o "$OUT/obj/$f.o" 2>/dev/null &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 "$OUT/obj/dsort_wave.o" "$OUT/obj/dsort_text.o" "$OUT/obj/dsort_api.o" -shared -L/opt/rocm/lib -lrccl -lrocprofiler-sdk-roctx \
  -Wl,-rpath,/opt/rocm/lib -lamdhip64 -o "$OUT/libdsort.so"
echo "built $OUT/libdsort.so"
