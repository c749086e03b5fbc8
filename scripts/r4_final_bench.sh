#!/bin/bash
# Round-4 final: the default bench line as the driver runs it (DEV TOOL)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r4_default_bench_e.json 2> gpurun_out/r4_default_bench_e.err
