#!/bin/bash
# Round-5 profile set, part b (run on the GPU box): the default bench line as the driver runs it, config
# 4's frame on one GPU, and the per-rank shares of configs 3 and 4 (multi-GPU projection).  (The
# triangle pre-filter's full-size A/B, base vs RT_TRI_FILTER=0, ran here before: r5_mesh50k_ab.log.)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r5_default_bench.json 2> gpurun_out/r5_default_bench.err || exit $?
timeout -k 10 300 python3 bench.py --config rtow4k --steps 3 --warmup 1 --no-cpu-baseline --no-end-to-end --no-pmc > gpurun_out/r5_rtow4k_bench.json 2> gpurun_out/r5_rtow4k_bench.err || exit $?
timeout -k 10 300 python3 scripts/share_sweep.py --reps 3 > gpurun_out/r5_shares.json 2> gpurun_out/r5_shares.err || exit $?
