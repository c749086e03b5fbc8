#!/bin/bash
# Round-4 A/B set l (DEV TOOL): the sphere roots' divisions by a = d.d as Markstein corrections
# (RT_ROOT_RCP=1) vs IEEE divisions (0)
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r4_ab_l.log
timeout -k 10 300 bash scripts/ab_lib.sh "rtow 256 f64" rcp0 rcp1 > $L 2>&1 || exit 1
timeout -k 10 300 bash scripts/ab_lib.sh "rtow 256 f64" rcp0 rcp1 >> $L 2>&1 || exit 1
timeout -k 10 300 bash scripts/ab_lib.sh "rtow 256 f32" rcp0 rcp1 >> $L 2>&1 || exit 1
