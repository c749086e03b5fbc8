#!/bin/bash
# mesh50k progressive (DEV TOOL): one batch vs 16 fused batches of 16 spp (config 5: 256 spp), default chunk rule and
# RT_POOL_CHUNK overrides (the fused batches take min(chunk, batch) balanced over the batch)
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r5_mesh_progress.log
: > $L
for c in default 8 16 default; do
  echo "== chunk $c" >> $L
  if [ $c = default ]; then
    PROBE_CONFIG=mesh50k timeout -k 10 200 python3 scripts/probe_progressive.py 3 0,16 >> $L 2>&1 || exit 1
  else
    RT_POOL_CHUNK=$c PROBE_CONFIG=mesh50k timeout -k 10 200 python3 scripts/probe_progressive.py 3 0,16 >> $L 2>&1 || exit 1
  fi
done
