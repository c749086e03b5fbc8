#!/bin/bash
# Round 5 A/B (DEV TOOL): normalize's min3 guard + the leave rule binary64-only (new) vs before (cur) vs
# new with the provable two-correction binary64 divisions (dv2) vs round 4
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r5_ab_i.log
: > $L
for rep in 1 2; do
  for v in new cur dv2 r4; do
    for w in "cornell 512 f64" "rtow 256 f32" "rtow 256 f64"; do
      echo -n "$v: " >> $L
      RT_HIP_LIB=blenderraytracer_amd/lib/variants/$v.so timeout -k 10 120 python3 scripts/probe_speed.py $w 2>&1 | grep Msamples >> $L || exit 1
    done
  done
done
