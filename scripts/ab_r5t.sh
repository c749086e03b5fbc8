#!/bin/bash
# Round 5 A/B (DEV TOOL): flags for the one-wave translation unit only (on top of the trackers): early
# if-conversion, relaxed occupancy scheduling, metric bias 30, no unclustered high-RP rescheduling
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r5_ab_t.log
: > $L
for rep in 1 2; do
  for v in base owifc owrel owb30 ownhrp; do
    for w in "mesh50k 256 f64" "cornell 512 f64"; do
      echo -n "$v: " >> $L
      RT_HIP_LIB=blenderraytracer_amd/lib/variants/$v.so timeout -k 10 120 python3 scripts/probe_speed.py $w 2>&1 | grep Msamples >> $L || exit 1
    done
  done
done
