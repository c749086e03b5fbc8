#!/bin/bash
# Progressive-render diagnosis (DEV TOOL): 16 fused batches of config 3 from Python without / with a progress
# callback / with callback and previews, for the current library, round 4's and the fence-free one
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r5_progress_diag.log
: > $L
for v in cur r4 fence0 cur r4; do
  lib=blenderraytracer_amd/lib/librt_hip.so; [ $v != cur ] && lib=blenderraytracer_amd/lib/variants/$v.so
  for mode in none progress preview; do
    e=""; [ $mode != none ] && e="PROBE_PROGRESS=1"; [ $mode = preview ] && e="$e PROBE_PREVIEW=1"
    echo "== $v $mode" >> $L
    env $e RT_HIP_LIB=$lib timeout -k 10 200 python3 scripts/probe_progressive.py 3 32 >> $L 2>&1 || exit 1
  done
done
