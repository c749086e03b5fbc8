#!/bin/bash
# Kernel timeline of a 16-batch progressive render with previews (DEV TOOL): config 3, one fused launch
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/tl
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tl/fused -o run -- python3 scripts/probe_preview_timeline.py 2 1 > gpurun_out/tl/fused.log 2>&1 || exit 1
