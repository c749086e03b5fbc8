#!/bin/bash
# Round-5 A/B set c (DEV TOOL): the fused commit protocol (fence0 = round 4's s_waitcnt form, base = one
# release fence per item, fence2 = acq_rel RMW), binary64 divisions (div1 = one Markstein correction,
# base = two, divoff = IEEE divisions), and the longest-first tile order on the last chunk only
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r5_ab_c.log
: > $L
for v in base fence0 fence2 fence2 fence0 base; do
  echo "== $v" >> $L
  RT_HIP_LIB=blenderraytracer_amd/lib/variants/$v.so timeout -k 10 200 python scripts/probe_progressive.py 3 0,32 >> $L 2>&1 || exit 1
done
timeout -k 10 300 bash scripts/ab_lib.sh "rtow 256 f64" base div1 divoff >> $L 2>&1 || exit 1
for v in 3 0 0 3; do
  echo "== RT_TILE_LPT=$v" >> $L
  RT_TILE_LPT=$v timeout -k 10 240 python scripts/share_sweep.py --reps 3 > gpurun_out/r5_shares_c_lpt$v.json 2>> $L || exit 1
done
