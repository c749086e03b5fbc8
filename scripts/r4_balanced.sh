#!/bin/bash
# Balanced chunks within progressive batches (DEV TOOL): the batch / cancel / resume GPU tests, then the
# progressive cost on mesh50k (16 x 16 spp) and config 3 (16 x 32 spp)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_js_host.py -m gpu -x -v --timeout 200 --timeout-method thread \
  -k "progressive or overlapped or cancel or resume or checkpoint or multi_device or js_gpu or sharded" > gpurun_out/r4_balanced_tests.log 2>&1 || exit 1
L=gpurun_out/r4_balanced.log
: > $L
for c in mesh50k rtow; do
  echo "== $c" >> $L
  PROBE_CONFIG=$c timeout -k 10 200 python scripts/probe_progressive.py 3 0,16,32 >> $L 2>&1 || exit 1
done
