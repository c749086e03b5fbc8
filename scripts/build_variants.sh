#!/bin/bash
# Builds librt_hip.so variants for A/B runs into blenderraytracer_amd/lib/variants/<name>.so.
# usage: scripts/build_variants.sh name:"-DFLAG=1 -DOTHER=2" ...
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/blenderraytracer_amd/lib/variants
mkdir -p "$OUT"
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fPIC $flags -I "$ROOT/include" \
    -c "$ROOT/blenderraytracer_amd/csrc/pt_trace.hip" -o "$OUT/$name.trace.o" &
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fPIC $flags -I "$ROOT/include" \
    -c "$ROOT/blenderraytracer_amd/csrc/rt_capi.cpp" -o "$OUT/$name.capi.o" &
  wait
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$OUT/$name.so" "$OUT/$name.trace.o" "$OUT/$name.capi.o"
  rm -f "$OUT/$name.trace.o" "$OUT/$name.capi.o"
  echo "built $OUT/$name.so ($flags)"
done
