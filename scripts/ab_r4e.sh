#!/bin/bash
# Round-4 A/B set e (DEV TOOL): Dielectric's 1/ior and r0 precomputed (dielpre) vs cur; deferred
# dielectric shading (dd4 / dd8); divisions by one scalar through Markstein corrections (divrcp).
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r4_ab_e.log
timeout -k 10 250 bash scripts/ab_lib.sh "rtow 256 f64" cur dielpre divrcp > $L 2>&1 || exit 1
timeout -k 10 250 bash scripts/ab_lib.sh "rtow 256 f64" dielpre dd4 dd8 >> $L 2>&1 || exit 1
timeout -k 10 250 bash scripts/ab_lib.sh "rtow 256 f32" cur dielpre divrcp >> $L 2>&1 || exit 1
timeout -k 10 250 bash scripts/ab_lib.sh "mesh50k 64 f64" dielpre divrcp >> $L 2>&1 || exit 1
