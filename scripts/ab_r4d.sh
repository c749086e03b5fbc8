#!/bin/bash
# Round-4 A/B set d (DEV TOOL): grid entry cell through the reciprocal in binary64 too (div2), the grid
# LDS kernel at 6 waves/SIMD (w6).
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r4_ab_d.log
timeout -k 10 250 bash scripts/ab_lib.sh "rtow 256 f64" cur div2 w6 > $L 2>&1 || exit 1
timeout -k 10 200 bash scripts/ab_lib.sh "rtow 256 f64" cur nodiel >> $L 2>&1 || exit 1
