#!/bin/bash
# Round-4 A/B set k (DEV TOOL): mesh50k pool chunk with XCD-contiguous item runs (rule 12)
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r4_ab_k.log
timeout -k 10 400 bash scripts/chunk_env_ab.sh "mesh50k 256 f64" 0 8 16 24 > $L 2>&1 || exit 1
