#!/bin/bash
# Builds librt_hip.so variants for A/B runs into blenderraytracer_amd/lib/variants/<name>.so.
# usage: scripts/build_variants.sh name:"-DFLAG=1 -DOTHER=2" ...
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/blenderraytracer_amd/lib/variants
SRCS="pt_trace.hip pt_onewave.hip rt_capi.cpp scene_json.cpp"   # the same sources (and per-source flags) as build.py
mkdir -p "$OUT"
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  objs=""
  for src in $SRCS; do
    obj="$OUT/$name.${src%.*}.o"
    extra=""; [ $src = pt_onewave.hip ] && [ -z "$NO_TRK" ] && extra="-mllvm -amdgpu-use-amdgpu-trackers=1"
    [ $src = pt_onewave.hip ] && extra="$extra $EXTRA_OW"   # (A/B: flags for the one-wave TU only)
    /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fPIC -mllvm -structurizecfg-skip-uniform-regions=1 $extra $flags -I "$ROOT/include" \
      -c "$ROOT/blenderraytracer_amd/csrc/$src" -o "$obj" &
    objs="$objs $obj"
  done
  wait
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$OUT/$name.so" $objs
  rm -f $objs
  echo "built $OUT/$name.so ($flags)"
done
