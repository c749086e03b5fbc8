#!/bin/bash
# Round 5 A/B (DEV TOOL): bisect the Cornell / f32 / f64 gap to round 4 with compile-time toggles (r4eq: every
# round-5 toggle at its round-4 setting; f0: the commit fence only; r4eqd: all but the divisions)
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r5_ab_j.log
: > $L
for rep in 1 2; do
  for v in new r4eq f0 r4eqd r4; do
    for w in "cornell 512 f64" "rtow 256 f32" "rtow 256 f64"; do
      echo -n "$v: " >> $L
      RT_HIP_LIB=blenderraytracer_amd/lib/variants/$v.so timeout -k 10 120 python3 scripts/probe_speed.py $w 2>&1 | grep Msamples >> $L || exit 1
    done
  done
done
