#!/bin/bash
# Round 5 A/B (DEV TOOL): more LLVM AMDGPU codegen options for the whole library — wave priority in VALU
# sections, early if-conversion, preallocated SGPR-spill VGPRs, no unclustered high-RP rescheduling
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r5_ab_s.log
: > $L
for rep in 1 2; do
  for v in base wprio ifcvt presgpr nohrp; do
    [ -f blenderraytracer_amd/lib/variants/$v.so ] || continue
    for w in "rtow 256 f64" "rtow 256 f32" "mesh50k 256 f64" "cornell 512 f64"; do
      echo -n "$v: " >> $L
      RT_HIP_LIB=blenderraytracer_amd/lib/variants/$v.so timeout -k 10 120 python3 scripts/probe_speed.py $w 2>&1 | grep Msamples >> $L || exit 1
    done
  done
done
