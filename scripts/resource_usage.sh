#!/bin/bash
# gfx950 resource usage of the trace kernels at this tree (compiler remarks, DEV TOOL): prints the
# pool kernels' VGPRs, spills, scratch, occupancy and LDS.  usage: bash scripts/resource_usage.sh > out.txt
ROOT=$(cd "$(dirname "$0")/.." && pwd)
echo "# hipcc -O3 -Rpass-analysis=kernel-resource-usage on csrc/pt_trace.hip ($(git -C $ROOT rev-parse --short HEAD 2>/dev/null))"
echo "# trace_pool_kernel<R, COUNT, ACC>: ACC 0 brute force, 2 stackless BVH, 3 ordered BVH walk, 4 its sphere-only form; trace_pool_lds_kernel<R, COUNT>: 4 with the nodes in LDS"
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fPIC -mllvm -structurizecfg-skip-uniform-regions=1 \
  -I "$ROOT/include" -c "$ROOT/blenderraytracer_amd/csrc/pt_trace.hip" -o /tmp/resource_usage.o -Rpass-analysis=kernel-resource-usage 2>&1 \
  | sed 's/^.*remark: *//; s/ \[-Rpass-analysis=kernel-resource-usage\]//' \
  | awk '/^Function Name:/ {keep = ($3 ~ /trace_pool(_lds)?_kernel/)} keep && /Function Name|VGPRs:|VGPRs Spill|SGPRs Spill|ScratchSize|Occupancy|LDS Size/'
