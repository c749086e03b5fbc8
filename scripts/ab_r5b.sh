#!/bin/bash
# Round-5 A/B set b (DEV TOOL): the longest-first tile order (RT_TILE_LPT=1, default) against raster order
# (0) on the per-rank shares of configs 3 and 4 (scripts/share_sweep.py) and the full config-3 frame
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r5_ab_b.log
: > $L
for v in 1 0 0 1; do
  echo "== RT_TILE_LPT=$v" >> $L
  RT_TILE_LPT=$v timeout -k 10 240 python scripts/share_sweep.py --reps 3 > gpurun_out/r5_shares_lpt$v.json 2>> $L || exit 1
  RT_TILE_LPT=$v timeout -k 10 120 python scripts/probe_speed.py rtow 512 f64 >> $L 2>&1 || exit 1
done
