#!/bin/bash
# Round-4 A/B set p (DEV TOOL): deferred regeneration threshold re-measured on the final kernel
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r4_ab_p.log
timeout -k 10 300 bash scripts/ab_lib.sh "rtow 256 f64" d12 d16 d20 > $L 2>&1 || exit 1
timeout -k 10 300 bash scripts/ab_lib.sh "rtow 256 f64" d12 d16 d20 >> $L 2>&1 || exit 1
