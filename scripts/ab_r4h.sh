#!/bin/bash
# Round-4 A/B set h (DEV TOOL): pool chunk at the per-rank shares of config 3 (64 / 128 spp per rank at
# N = 8 / 4): the rule vs smaller chunks (shorter drain tail, more partials)
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r4_ab_h.log
timeout -k 10 250 bash scripts/chunk_env_ab.sh "rtow 64 f64" 0 6 8 11 > $L 2>&1 || exit 1
timeout -k 10 250 bash scripts/chunk_env_ab.sh "rtow 128 f64" 0 11 16 >> $L 2>&1 || exit 1
timeout -k 10 250 bash scripts/chunk_env_ab.sh "rtow 512 f64" 0 32 64 90 >> $L 2>&1 || exit 1
