#!/bin/bash
# Round-4 A/B set q (DEV TOOL): preview frames in binary32 arithmetic (pv32) vs binary64 mean and tone
# map (pv64): config 3 in 16 fused batches with a preview frame at every progress call
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r4_ab_q.log
: > $L
for v in pv64 pv32 pv32 pv64; do
  echo "== $v" >> $L
  RT_HIP_LIB=blenderraytracer_amd/lib/variants/$v.so timeout -k 10 200 python scripts/probe_preview_timeline.py 3 1 >> $L 2>&1 || exit 1
done
