#!/bin/bash
# rocprofv3 evidence for one bench workload (run on the GPU box from the repo root):
#   1. kernel trace + stats of the bench command (bench's own counter passes off: no nested profiler)
#   2. the bench line itself, whose roofline comes from its own FETCH_SIZE / WRITE_SIZE / SQ passes
#      (kept: their counter CSVs are copied next to the trace)
# usage: bash scripts/profile_round.sh <tag> <bench args...>   -> gpurun_out/prof_<tag>/...
set -o pipefail
tag=$1; shift
out=gpurun_out/prof_$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -o run -- python3 bench.py --no-cpu-baseline --no-pmc "$@" > $out/bench_under_trace.log 2>&1 || exit $?
BENCH_PMC_KEEP=$out/pmc timeout -k 10 600 python3 bench.py --no-cpu-baseline --no-end-to-end "$@" > $out/bench.json 2> $out/bench.err || exit $?
tail -1 $out/bench.json
