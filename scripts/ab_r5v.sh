#!/bin/bash
# Round 5 A/B (DEV TOOL): the binary64 grid LDS kernel at 6 / 4 waves per SIMD vs 5 on the final code
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r5_ab_v.log
: > $L
for rep in 1 2 3; do
  for v in base g6 g4; do
    echo -n "$v: " >> $L
    RT_HIP_LIB=blenderraytracer_amd/lib/variants/$v.so timeout -k 10 120 python3 scripts/probe_speed.py rtow 256 f64 2>&1 | grep Msamples >> $L || exit 1
  done
done
