#!/bin/bash
# Round 5 A/B (DEV TOOL): the one-wave kernels in their own translation unit with LLVM's register-pressure
# trackers (tu) vs the same split without them (notrk), all four workloads; then the GPU test suite
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r5_ab_r.log
: > $L
for rep in 1 2; do
  for v in tu notrk; do
    for w in "rtow 256 f64" "rtow 256 f32" "mesh50k 256 f64" "cornell 512 f64"; do
      echo -n "$v: " >> $L
      RT_HIP_LIB=blenderraytracer_amd/lib/variants/$v.so timeout -k 10 120 python3 scripts/probe_speed.py $w 2>&1 | grep Msamples >> $L || exit 1
    done
  done
done
timeout -k 10 900 python3 -u -m pytest tests/ -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r5_tu_tests.log 2>&1 || exit 1
