#!/bin/bash
# Round 5 A/B (DEV TOOL): LLVM AMDGPU scheduler strategies for the whole library — max-ilp, max-memory-clause,
# the AMDGPU register-pressure trackers — against the default, on all four workloads
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r5_ab_q.log
: > $L
for rep in 1 2; do
  for v in base ilp mclause trk; do
    [ -f blenderraytracer_amd/lib/variants/$v.so ] || continue
    for w in "rtow 256 f64" "rtow 256 f32" "mesh50k 256 f64" "cornell 512 f64"; do
      echo -n "$v: " >> $L
      RT_HIP_LIB=blenderraytracer_amd/lib/variants/$v.so timeout -k 10 120 python3 scripts/probe_speed.py $w 2>&1 | grep Msamples >> $L || exit 1
    done
  done
done
