#!/bin/bash
# Round 5 A/B (DEV TOOL): the binary64 grid walk's sphere filter two records per packed instruction (pk)
# vs one record at a time (pk0), RTOW f64 (images must be identical)
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r5_ab_l.log
: > $L
for rep in 1 2 3; do
  for v in pk pk0; do
    echo -n "$v: " >> $L
    RT_HIP_LIB=blenderraytracer_amd/lib/variants/$v.so timeout -k 10 120 python3 scripts/probe_speed.py rtow 256 f64 2>&1 | grep Msamples >> $L || exit 1
  done
done
