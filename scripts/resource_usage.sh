#!/bin/bash
# gfx950 resource usage of the trace kernels at this tree (compiler remarks, DEV TOOL): prints the
# pool kernels' VGPRs, spills, scratch, occupancy and LDS.  usage: bash scripts/resource_usage.sh > out.txt
ROOT=$(cd "$(dirname "$0")/.." && pwd)
echo "# hipcc -O3 -Rpass-analysis=kernel-resource-usage on csrc/pt_trace.hip and pt_onewave.hip ($(git -C $ROOT rev-parse --short HEAD 2>/dev/null))"
echo "# trace_pool_kernel<R, COUNT, ACC, CANCEL>: ACC 0 brute force, 1 its lean form (spheres + planes), 2 stackless BVH, 3 ordered BVH walk, 10 its lean form (no boxes), 4 the sphere-only walk, 6 the grid; trace_pool_lds_kernel<R, COUNT, ACC>: 5 sphere-tree nodes in LDS, 7 the grid in LDS, 9 its lean form (spheres only), 8 triangle-tree top levels in LDS (opt-in); lean = sky gradient, perspective camera, supersampling only"
for src in pt_trace.hip pt_onewave.hip; do
  extra=""; [ $src = pt_onewave.hip ] && extra="-mllvm -amdgpu-use-amdgpu-trackers=1"   # as build.py
  echo "## $src $extra"
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fPIC -mllvm -structurizecfg-skip-uniform-regions=1 $extra \
    -I "$ROOT/include" -c "$ROOT/blenderraytracer_amd/csrc/$src" -o /tmp/resource_usage.o -Rpass-analysis=kernel-resource-usage 2>&1 \
    | sed 's/^.*remark: *//; s/ \[-Rpass-analysis=kernel-resource-usage\]//' \
    | awk '/^Function Name:/ {keep = ($3 ~ /trace_pool(_lds)?_kernel/)} keep && /Function Name|VGPRs:|VGPRs Spill|SGPRs Spill|ScratchSize|Occupancy|LDS Size/'
done
