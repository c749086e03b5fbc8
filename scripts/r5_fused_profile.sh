#!/bin/bash
# Round 5 (DEV TOOL): kernel trace of config 3 rendered as 16 fused progressive batches with running frames
# (one trace launch, no CANCEL instantiation since the queue-move cancel) under rocprofv3
set -o pipefail
mkdir -p gpurun_out/prof_fused
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
PROBE_PREVIEW=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fused -o run -- python3 scripts/probe_progressive.py 2 32 > gpurun_out/prof_fused/probe.log 2>&1 || exit 1
