#!/bin/bash
# Round-4 final profile set d: RTOW f32 (Markstein roots) under rocprofv3 + the bench's counter passes,
# then the default bench line as the driver runs it.
set -o pipefail
bash scripts/profile_round.sh rtow_f32 --config rtow --precision f32 --steps 10 --warmup 2 || exit $?
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r4_default_bench_d.json 2> gpurun_out/r4_default_bench_d.err
