#!/bin/bash
# (DEV TOOL) the resume / concurrent-cancel tests with their diagnostics, then the GPU suite
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -v -s --timeout 250 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "two_concurrent or one_batch_left or checkpoint_resume" > gpurun_out/r5_two_diag.log 2>&1 || exit 1
timeout -k 10 900 python3 -u -m pytest tests/ -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r5_tu_tests.log 2>&1 || exit 1
