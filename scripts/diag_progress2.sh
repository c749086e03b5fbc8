#!/bin/bash
# Progressive-render bisection (DEV TOOL): 16 fused batches and one batch of config 3 for the current
# library and variants that undo one round-5 change each (binary64 divisions, the dominant spheres' leave rule)
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r5_progress_diag2.log
: > $L
for v in base r4 c_6ed14f4 c_4b6b48f divtw div1 awayold base r4 c_6ed14f4 c_4b6b48f divtw; do
  echo "== $v" >> $L
  RT_HIP_LIB=blenderraytracer_amd/lib/variants/$v.so timeout -k 10 200 python3 scripts/probe_progressive.py 3 0,32 >> $L 2>&1 || exit 1
done
