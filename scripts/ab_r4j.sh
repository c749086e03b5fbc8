#!/bin/bash
# Round-4 A/B set j (DEV TOOL): pool chunk above the rule at the per-rank shares of config 3 (64 / 128
# spp per rank at N = 8 / 4): fewer, longer items
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r4_ab_j.log
timeout -k 10 250 bash scripts/chunk_env_ab.sh "rtow 64 f64" 0 22 32 > $L 2>&1 || exit 1
timeout -k 10 250 bash scripts/chunk_env_ab.sh "rtow 128 f64" 0 32 43 >> $L 2>&1 || exit 1
timeout -k 10 250 bash scripts/chunk_env_ab.sh "rtow 256 f64" 0 >> $L 2>&1 || exit 1
