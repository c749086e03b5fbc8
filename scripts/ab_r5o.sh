#!/bin/bash
# Round 5 A/B (DEV TOOL): the camera's words reloaded from the kernel-argument segment at each sample
# start (camr) vs kept live in SGPRs (camr0), on all four workloads (images must be identical)
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r5_ab_o.log
: > $L
for rep in 1 2; do
  for v in camr camr0; do
    for w in "rtow 256 f64" "rtow 256 f32" "mesh50k 256 f64" "cornell 512 f64"; do
      echo -n "$v: " >> $L
      RT_HIP_LIB=blenderraytracer_amd/lib/variants/$v.so timeout -k 10 120 python3 scripts/probe_speed.py $w 2>&1 | grep Msamples >> $L || exit 1
    done
  done
done
