#!/bin/bash
# Round 5 (DEV TOOL): the one-wave pool's progressive renders on per-XCD queues (trace_pool_xcd_kernel,
# cancel by moving the queues) vs the CANCEL instantiation (xq0); one-shot frames forced through the
# XCD kernel (RT_XCD_QUEUES_ALL=1) vs the one-wave kernel; then the progressive/cancel GPU tests, the
# fused stress, and the one-shot parity tests with every one-wave launch on the XCD kernel
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r5_xcd_queues.log
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
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_js_host.py \
  -k "cancel or resume or progress or overlap or preview or multi_device or checkpoint" > gpurun_out/r5_xcd_tests.log 2>&1 || exit 1
timeout -k 10 400 python3 -u scripts/stress_fused.py 120 > gpurun_out/r5_xcd_stress.log 2>&1 || exit 1
RT_XCD_QUEUES_ALL=1 timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "mesh or cornell or brute or bvh or golden or oracle" > gpurun_out/r5_xcd_forced_tests.log 2>&1 || exit 1
