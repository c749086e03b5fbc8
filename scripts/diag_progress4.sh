#!/bin/bash
# Progressive-render diagnosis 4 (DEV TOOL): one batch and 16 fused batches of config 3 for variants of the
# CANCEL kernel's polling (pos: by queue position) and of the binary64 divisions (dv: round 4's form)
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r5_progress_diag4.log
: > $L
for v in base pos dv posdv r4 base pos dv posdv r4; do
  echo "== $v" >> $L
  RT_HIP_LIB=blenderraytracer_amd/lib/variants/$v.so timeout -k 10 200 python3 scripts/probe_progressive.py 3 0,32 >> $L 2>&1 || exit 1
done
