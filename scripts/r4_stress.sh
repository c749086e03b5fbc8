#!/bin/bash
# Fused-batch stress on the GPU (DEV TOOL)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u scripts/stress_fused.py 150 > gpurun_out/r4_stress.log 2>&1
