#!/bin/bash
# Fused progressive batches (DEV TOOL): the progressive / batch / cancel GPU tests, then the 16-batch
# cost with and without the fused launch, then the one-batch headline against the previous sources
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r4_fused.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_js_host.py -m gpu -x -v --timeout 200 --timeout-method thread \
  -k "progressive or overlapped or cancel or resume or checkpoint or multi_device or js_gpu or sharded" > gpurun_out/r4_fused_tests.log 2>&1 || exit 1
echo "== fused (default)" > $L
timeout -k 10 200 python scripts/probe_progressive.py 3 0,32,64 >> $L 2>&1 || exit 1
echo "== RT_FUSED_BATCHES=0" >> $L
RT_FUSED_BATCHES=0 timeout -k 10 200 python scripts/probe_progressive.py 3 0,32 >> $L 2>&1 || exit 1
timeout -k 10 250 bash scripts/ab_lib.sh "rtow 512 f64" head fused >> $L 2>&1 || exit 1
