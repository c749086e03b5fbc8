#!/bin/bash
# Progressive-render diagnosis 6 (DEV TOOL): cancel by moving the queue past the last item (bump) vs
# round 4's wave-0 poll + LDS stop flag (old) vs round 4, one batch and 16 fused batches of config 3
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r5_progress_diag6.log
: > $L
for v in bump old r4 bump old r4; do
  echo "== $v" >> $L
  RT_HIP_LIB=blenderraytracer_amd/lib/variants/$v.so timeout -k 10 200 python3 scripts/probe_progressive.py 3 0,32 >> $L 2>&1 || exit 1
done
