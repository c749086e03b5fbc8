#!/bin/bash
# Round-4 profile set c (fused progressive batches, XCD-contiguous item runs): headline RTOW f64 and
# mesh50k under rocprofv3 + the bench's counter passes, then the default bench line as the driver runs it.
set -o pipefail
bash scripts/profile_round.sh rtow_f64 --config rtow --precision f64 --steps 10 --warmup 2 || exit $?
bash scripts/profile_round.sh mesh50k_f64 --config mesh50k --precision f64 --steps 5 --warmup 1 || exit $?
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r4_default_bench.json 2> gpurun_out/r4_default_bench.err
