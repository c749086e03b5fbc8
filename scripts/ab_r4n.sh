#!/bin/bash
# Round-4 probe n (DEV TOOL): progressive cost on mesh50k and Cornell (one-wave pool kernel: every
# workgroup reads the cancel word) with and without the reads (nopoll.so)
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r4_ab_n.log
: > $L
for c in mesh50k cornell; do
  for v in "" "RT_HIP_LIB=blenderraytracer_amd/lib/variants/nopoll.so"; do
    echo "== $c $v" >> $L
    env PROBE_CONFIG=$c $v timeout -k 10 200 python scripts/probe_progressive.py 3 0,16 >> $L 2>&1 || exit 1
  done
done
