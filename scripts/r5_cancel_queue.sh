#!/bin/bash
# Round 5 (DEV TOOL): cancel by moving the LDS pool launches' queues (no cancel poll in the LDS kernel):
# config 3 one batch / 16 fused batches vs round 4, the fused stress, then the whole GPU test suite
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r5_cancel_queue.log
: > $L
for v in cur r4 cur r4; do
  echo "== $v" >> $L
  RT_HIP_LIB=blenderraytracer_amd/lib/variants/$v.so timeout -k 10 200 python3 scripts/probe_progressive.py 3 0,32 >> $L 2>&1 || exit 1
done
timeout -k 10 400 python3 -u scripts/stress_fused.py 120 > gpurun_out/r5_cancel_stress.log 2>&1 || exit 1
timeout -k 10 840 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/ > gpurun_out/r5_gpu_tests.log 2>&1 || exit 1
