#!/bin/bash
# Round-4 A/B set g (DEV TOOL): the pool's item visiting order — tiles in S x S blocks (tbS) and
# XCD-contiguous runs of K one-wave workgroups (xK) against raster order (base).
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r4_ab_g3.log
timeout -k 10 500 bash scripts/ab_lib.sh "mesh50k 256 f64" base tb8x1024 tb8x2048 tb4x1024 x1024 > $L 2>&1 || exit 1
timeout -k 10 200 bash scripts/ab_lib.sh "cornell 64 f64" base tb8x1024 >> $L 2>&1 || exit 1
