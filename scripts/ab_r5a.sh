#!/bin/bash
# Round-5 A/B set a (DEV TOOL): the binary32 triangle pre-filter (trif0 = off), binary64 divisions with
# one Markstein correction (div1) instead of two, and the fused-batch commit protocol without fences
# (fence0: round 4's s_waitcnt form), against the round-5 defaults (base)
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r5_ab_a.log
: > $L
timeout -k 10 300 bash scripts/ab_lib.sh "mesh50k 128 f64" base trif0 >> $L 2>&1 || exit 1
timeout -k 10 300 bash scripts/ab_lib.sh "mesh50k 128 f64" base trif0 >> $L 2>&1 || exit 1
timeout -k 10 300 bash scripts/ab_lib.sh "rtow 256 f64" base div1 >> $L 2>&1 || exit 1
timeout -k 10 300 bash scripts/ab_lib.sh "rtow 256 f64" base div1 >> $L 2>&1 || exit 1
for v in base fence0 base fence0; do
  echo "== $v" >> $L
  RT_HIP_LIB=blenderraytracer_amd/lib/variants/$v.so timeout -k 10 200 python scripts/probe_progressive.py 3 0,32 >> $L 2>&1 || exit 1
done
