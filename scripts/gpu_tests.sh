#!/bin/bash
# The GPU test tier as the driver runs it, plus smoke() (run on the GPU box from the repo root).
# usage: bash scripts/gpu_tests.sh <tag>   -> gpurun_out/<tag>_tests.log, gpurun_out/<tag>_smoke.log
set -o pipefail
tag=${1:-gpu}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1
