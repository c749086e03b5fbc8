#!/bin/bash
# Round 5 A/B (DEV TOOL): vdiv_rcp guard as one min3 + one max3 (mm) vs the min3 normalize guard only
# (new) vs round 4
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r5_ab_k.log
: > $L
for rep in 1 2; do
  for v in mm new r4; do
    for w in "cornell 512 f64" "rtow 256 f32" "rtow 256 f64"; do
      echo -n "$v: " >> $L
      RT_HIP_LIB=blenderraytracer_amd/lib/variants/$v.so timeout -k 10 120 python3 scripts/probe_speed.py $w 2>&1 | grep Msamples >> $L || exit 1
    done
  done
done
