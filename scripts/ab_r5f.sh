#!/bin/bash
# Round-5 A/B set f (DEV TOOL): (double)width / height recomputed at every sample start (opwh) instead of
# hoisted into scratch by the compiler (base)
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r5_ab_f.log
: > $L
for w in "rtow 256 f64" "rtow 256 f64" "rtow 256 f32" "mesh50k 64 f64"; do
  timeout -k 10 300 bash scripts/ab_lib.sh "$w" base opwh >> $L 2>&1 || exit 1
done
