#!/bin/bash
# Round-4 A/B set c (DEV TOOL): grid density after the survivor masks (RTOW f64 / f32).
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r4_ab_c.log
echo "-- grid density f64" > $L
timeout -k 10 250 bash scripts/ab_lib.sh "rtow 256 f64" cur lam0125 lam009 lam0063 >> $L 2>&1 || exit 1
echo "-- grid density f32" >> $L
timeout -k 10 200 bash scripts/ab_lib.sh "rtow 256 f32" cur lam0125 lam009 >> $L 2>&1 || exit 1
echo "-- dominant spheres through survivor masks (bigc) vs per sphere (cur)" >> $L
timeout -k 10 200 bash scripts/ab_lib.sh "rtow 256 f64" cur bigc >> $L 2>&1 || exit 1
timeout -k 10 200 bash scripts/ab_lib.sh "mesh50k 64 f64" cur bigc >> $L 2>&1 || exit 1
