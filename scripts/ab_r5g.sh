#!/bin/bash
# Round-5 A/B set g (DEV TOOL): Dielectric.scatter out of line (cdiel: its registers leave the trace
# kernel's allocation) vs inline (base)
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r5_ab_g.log
: > $L
for w in "rtow 256 f64" "rtow 256 f64" "rtow 256 f32" "mesh50k 64 f64"; do
  timeout -k 10 300 bash scripts/ab_lib.sh "$w" base cdiel >> $L 2>&1 || exit 1
done
