#!/bin/bash
# Round-4 probe o (DEV TOOL): mesh50k in 16 batches of 16 spp: the chunk of each batch (rule: min(12, 16)
# = 12, i.e. chunks of 12 + 4) vs 8 (8 + 8) vs 16 (one chunk)
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r4_ab_o.log
: > $L
for c in 0 8 16; do
  echo "== RT_POOL_CHUNK=$c" >> $L
  if [ $c = 0 ]; then PROBE_CONFIG=mesh50k timeout -k 10 200 python scripts/probe_progressive.py 3 16 >> $L 2>&1 || exit 1
  else RT_POOL_CHUNK=$c PROBE_CONFIG=mesh50k timeout -k 10 200 python scripts/probe_progressive.py 3 16 >> $L 2>&1 || exit 1; fi
done
