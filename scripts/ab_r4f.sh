#!/bin/bash
# Round-4 A/B set f (DEV TOOL): the camera ray's (i + r) / width through RN(1 / width) (uv1) vs the
# divisions (uv0).
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r4_ab_f.log
timeout -k 10 250 bash scripts/ab_lib.sh "rtow 256 f64" uv0 uv1 > $L 2>&1 || exit 1
timeout -k 10 250 bash scripts/ab_lib.sh "cornell 64 f64" uv0 uv1 >> $L 2>&1 || exit 1
