#!/bin/bash
# Round 5 checkpoint (DEV TOOL): the driver's round-end sequence on the current tree — the GPU test
# suite, smoke(), the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests/ -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r5c_gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5c_smoke.log 2>&1 || exit 1
timeout -k 10 600 python3 bench.py > gpurun_out/r5c_bench.json 2> gpurun_out/r5c_bench.err || exit 1
