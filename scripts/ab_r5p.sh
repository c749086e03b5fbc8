#!/bin/bash
# Round 5 A/B (DEV TOOL): the reduce / preview side kernels looping over their tiles in at most 4096
# (sg) / 1024 (sg1k) one-wave workgroups vs one workgroup per tile (sg0); config 3 one batch and 16
# fused batches with running frames
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r5_ab_p.log
: > $L
for v in sg sg0 sg1k sg sg0 sg1k; do
  echo "== $v" >> $L
  PROBE_PREVIEW=1 RT_HIP_LIB=blenderraytracer_amd/lib/variants/$v.so timeout -k 10 200 python3 scripts/probe_progressive.py 3 0,32 >> $L 2>&1 || exit 1
done
