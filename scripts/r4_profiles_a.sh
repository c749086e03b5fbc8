#!/bin/bash
# Round-4 profile set, part a (run on the GPU box): headline RTOW f64 and f32 under rocprofv3
# (kernel trace + the bench's own counter passes), then config 4's frame on one GPU.
set -o pipefail
bash scripts/profile_round.sh rtow_f64 --config rtow --precision f64 --steps 10 --warmup 2 || exit $?
bash scripts/profile_round.sh rtow_f32 --config rtow --precision f32 --steps 10 --warmup 2 || exit $?
timeout -k 10 300 python3 bench.py --config rtow4k --steps 3 --warmup 1 --no-cpu-baseline --no-end-to-end --no-pmc > gpurun_out/r4_rtow4k_bench.json 2> gpurun_out/r4_rtow4k_bench.err
