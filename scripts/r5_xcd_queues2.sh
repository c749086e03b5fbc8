#!/bin/bash
# Round 5 (DEV TOOL), second form (next position prefetched, counters on separate lines): per-XCD queues (trace_pool_xcd_kernel,
# cancel by moving the queues) vs the CANCEL instantiation (xq0); one-shot frames forced through the
# XCD kernel (RT_XCD_QUEUES_ALL=1) vs the one-wave kernel; then the progressive/cancel GPU tests, the
# fused stress, and the one-shot parity tests with every one-wave launch on the XCD kernel
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r5_xcd_queues2.log
: > $L
for v in base xq0 base xq0; do
  for c in mesh50k:16 cornell:32; do
    echo "== $v ${c%%:*}" >> $L
    lib=blenderraytracer_amd/lib/librt_hip.so; [ $v = xq0 ] && lib=blenderraytracer_amd/lib/variants/xq0.so
    RT_HIP_LIB=$lib PROBE_CONFIG=${c%%:*} timeout -k 10 200 python3 scripts/probe_progressive.py 3 0,${c##*:} >> $L 2>&1 || exit 1
  done
done
for rep in 1 2; do
  for f in 0 1; do
    for w in "mesh50k 256 f64" "cornell 512 f64"; do
      echo -n "all=$f: " >> $L
      RT_XCD_QUEUES_ALL=$f timeout -k 10 120 python3 scripts/probe_speed.py $w 2>&1 | grep Msamples >> $L || exit 1
    done
  done
done
