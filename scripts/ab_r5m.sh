#!/bin/bash
# Round 5 A/B (DEV TOOL): config 5 (mesh50k f64) occupancy of the triangle walk (3 / 4 / 5 waves per SIMD)
# and XCD run length (512 / 1024 / 2048) with the triangle pre-filter in place
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r5_ab_m.log
: > $L
for rep in 1 2; do
  for v in base w5 w3 xr512 xr2k; do
    echo -n "$v: " >> $L
    RT_HIP_LIB=blenderraytracer_amd/lib/variants/$v.so timeout -k 10 120 python3 scripts/probe_speed.py mesh50k 256 f64 2>&1 | grep Msamples >> $L || exit 1
  done
done
