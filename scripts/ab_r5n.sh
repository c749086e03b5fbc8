#!/bin/bash
# Round 5 A/B (DEV TOOL): occupancy re-check on the round-5 code — brute force (Cornell f64) at 5 / 6 / 7
# waves per SIMD, the binary32 grid kernel (RTOW f32) at 5 / 6 / 7
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r5_ab_n.log
: > $L
for rep in 1 2; do
  for v in base mw5 mw7; do
    echo -n "$v: " >> $L
    RT_HIP_LIB=blenderraytracer_amd/lib/variants/$v.so timeout -k 10 120 python3 scripts/probe_speed.py cornell 512 f64 2>&1 | grep Msamples >> $L || exit 1
  done
  for v in base gw5 gw7; do
    echo -n "$v: " >> $L
    RT_HIP_LIB=blenderraytracer_amd/lib/variants/$v.so timeout -k 10 120 python3 scripts/probe_speed.py rtow 256 f32 2>&1 | grep Msamples >> $L || exit 1
  done
done
