#!/bin/bash
# Round-5 profile set, part a (run on the GPU box): headline RTOW f64, mesh50k f64, RTOW f32 and Cornell f64
# under rocprofv3 (kernel trace + the bench's own counter passes)
set -o pipefail
bash scripts/profile_round.sh rtow_f64 --config rtow --precision f64 --steps 10 --warmup 2 || exit $?
bash scripts/profile_round.sh mesh50k_f64 --config mesh50k --precision f64 --steps 10 --warmup 2 || exit $?
bash scripts/profile_round.sh rtow_f32 --config rtow --precision f32 --steps 10 --warmup 2 || exit $?
bash scripts/profile_round.sh cornell_f64 --config cornell --precision f64 --steps 20 --warmup 3 || exit $?
