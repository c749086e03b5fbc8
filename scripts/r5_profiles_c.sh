#!/bin/bash
# Round-5 profile set, part c (run on the GPU box): mesh50k and Cornell after the one-wave kernels moved
# to their own translation unit (pt_onewave.hip, register-pressure trackers), and the default bench line
set -o pipefail
bash scripts/profile_round.sh mesh50k_f64 --config mesh50k --precision f64 --steps 10 --warmup 2 || exit $?
bash scripts/profile_round.sh cornell_f64 --config cornell --precision f64 --steps 20 --warmup 3 || exit $?
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r5_default_bench.json 2> gpurun_out/r5_default_bench.err || exit $?
