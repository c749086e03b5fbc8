#!/bin/bash
# Round 5 A/B (DEV TOOL): where Cornell f64 and RTOW f32 lost against round 4 — current, round 4, round 4's
# single-correction binary64 divisions (dv1, unproven: measurement only), round 4's away rule (li0)
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r5_ab_h.log
: > $L
for rep in 1 2; do
  for v in cur r4 dv1 li0; do
    for w in "cornell 512 f64" "rtow 256 f32" "rtow 256 f64"; do
      echo -n "$v: " >> $L
      RT_HIP_LIB=blenderraytracer_amd/lib/variants/$v.so timeout -k 10 120 python3 scripts/probe_speed.py $w 2>&1 | grep Msamples >> $L || exit 1
    done
  done
done
