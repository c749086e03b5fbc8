#!/bin/bash
# Fused progressive batches A/B (DEV TOOL): 16 batches of 32 spp vs one batch, config 3: the LDS pool
# kernel's wave 0 reading the cancel word every 1 / 4 / 16 items, no reads (nopoll.so), and the
# previous sources (head.so, a launch per batch)
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r4_fused_ab3.log
: > $L
for v in every1 every4 every16 nopoll head; do
  echo "== $v" >> $L
  RT_HIP_LIB=blenderraytracer_amd/lib/variants/$v.so timeout -k 10 200 python scripts/probe_progressive.py 3 0,32 >> $L 2>&1 || exit 1
done
