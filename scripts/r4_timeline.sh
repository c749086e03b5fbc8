#!/bin/bash
# Kernel timeline of a 16-batch progressive render with previews (DEV TOOL)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/tl
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/tl/p1 -o run -- python3 scripts/probe_preview_timeline.py 2 1 > gpurun_out/tl/p1.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/tl/p0 -o run -- python3 scripts/probe_preview_timeline.py 2 0 > gpurun_out/tl/p0.log 2>&1 || exit 1
