#!/bin/bash
# Progressive-render diagnosis 3 (DEV TOOL): fused batches with and without the CANCEL kernel instantiation
# (RT_ITEM_CANCEL=0), for the current library and round 4's
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r5_progress_diag3.log
: > $L
for v in base r4 base r4; do
  for e in "" "RT_ITEM_CANCEL=0"; do
    echo "== $v $e" >> $L
    env $e RT_HIP_LIB=blenderraytracer_amd/lib/variants/$v.so timeout -k 10 200 python3 scripts/probe_progressive.py 3 32 >> $L 2>&1 || exit 1
  done
done
