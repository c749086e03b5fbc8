#!/bin/bash
# mesh50k progressive (DEV TOOL) 2: the fused launch without its cancel poll (RT_ITEM_CANCEL=0: the
# one-wave kernel's non-CANCEL instantiation), and the chunk rule's 12 inside 16-spp batches
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r5_mesh_progress2.log
: > $L
for v in base nocancel c12 base nocancel c12; do
  echo "== $v" >> $L
  case $v in
    base) PROBE_CONFIG=mesh50k timeout -k 10 200 python3 scripts/probe_progressive.py 3 0,16 >> $L 2>&1 || exit 1 ;;
    nocancel) RT_ITEM_CANCEL=0 PROBE_CONFIG=mesh50k timeout -k 10 200 python3 scripts/probe_progressive.py 3 0,16 >> $L 2>&1 || exit 1 ;;
    c12) RT_POOL_CHUNK=12 PROBE_CONFIG=mesh50k timeout -k 10 200 python3 scripts/probe_progressive.py 3 0,16 >> $L 2>&1 || exit 1 ;;
  esac
done
