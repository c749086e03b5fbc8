#!/bin/bash
# Progressive-render diagnosis 5 (DEV TOOL): the item body as a called function (ni) vs inlined (base)
# vs round 4, one batch and 16 fused batches of config 3, and the headline RTOW speed
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r5_progress_diag5.log
: > $L
for v in base ni r4 base ni r4; do
  echo "== $v" >> $L
  RT_HIP_LIB=blenderraytracer_amd/lib/variants/$v.so timeout -k 10 200 python3 scripts/probe_progressive.py 3 0,32 >> $L 2>&1 || exit 1
done
for v in base ni base ni; do
  echo -n "$v: " >> $L
  RT_HIP_LIB=blenderraytracer_amd/lib/variants/$v.so timeout -k 10 120 python3 scripts/probe_speed.py rtow 256 f64 2>&1 | grep Msamples >> $L || exit 1
done
