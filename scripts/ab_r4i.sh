#!/bin/bash
# Round-4 probe set i (DEV TOOL): where the 16-batch progressive render's cost goes — batch sizes, the
# cancel instantiation (RT_ITEM_CANCEL=0), overlapped batches off (RT_OVERLAP=0)
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r4_ab_i.log
echo "== default" > $L
timeout -k 10 200 python scripts/probe_progressive.py 3 0,32,64,128 >> $L 2>&1 || exit 1
echo "== RT_ITEM_CANCEL=0" >> $L
RT_ITEM_CANCEL=0 timeout -k 10 200 python scripts/probe_progressive.py 3 0,32 >> $L 2>&1 || exit 1
echo "== RT_OVERLAP=0" >> $L
RT_OVERLAP=0 timeout -k 10 200 python scripts/probe_progressive.py 3 0,32 >> $L 2>&1 || exit 1
