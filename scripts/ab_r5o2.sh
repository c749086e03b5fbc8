#!/bin/bash
# Round 5 A/B (DEV TOOL): the camera's words reloaded from the kernel-argument segment at each sample
# start in the binary32 LDS kernel only (camr, second form) vs every kernel keeping them (camr0)
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r5_ab_o2.log
: > $L
for rep in 1 2; do
  for v in camr camr0; do
    for w in "rtow 256 f64" "rtow 256 f32" "mesh50k 256 f64" "cornell 512 f64"; do
      echo -n "$v: " >> $L
      RT_HIP_LIB=blenderraytracer_amd/lib/variants/$v.so timeout -k 10 120 python3 scripts/probe_speed.py $w 2>&1 | grep Msamples >> $L || exit 1
    done
  done
done
