#!/bin/bash
# Round-5 A/B set e (DEV TOOL): the `leave` rule for every sphere (base) vs the dominant spheres only (leave0)
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r5_ab_e.log
: > $L
for w in "rtow 256 f64" "rtow 256 f64" "rtow 256 f32" "cornell 64 f64" "mesh50k 64 f64"; do
  timeout -k 10 300 bash scripts/ab_lib.sh "$w" base leave0 >> $L 2>&1 || exit 1
done
