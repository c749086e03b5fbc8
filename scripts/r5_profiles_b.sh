#!/bin/bash
# Round-5 profile set, part b (run on the GPU box): the default bench line as the driver runs it, config
# 4's frame on one GPU, and the per-rank shares of configs 3 and 4 (multi-GPU projection)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r5_default_bench.json 2> gpurun_out/r5_default_bench.err || exit $?
timeout -k 10 300 python3 bench.py --config rtow4k --steps 3 --warmup 1 --no-cpu-baseline --no-end-to-end --no-pmc > gpurun_out/r5_rtow4k_bench.json 2> gpurun_out/r5_rtow4k_bench.err || exit $?
timeout -k 10 300 python3 scripts/share_sweep.py --reps 3 > gpurun_out/r5_shares.json 2> gpurun_out/r5_shares.err || exit $?
# the triangle pre-filter at config 5's full size: the bench's trace step with (base) and without (trif0)
for v in base trif0 trif0 base; do
  RT_HIP_LIB=blenderraytracer_amd/lib/variants/$v.so timeout -k 10 300 python3 bench.py --config mesh50k --steps 5 --warmup 1 --no-cpu-baseline --no-end-to-end --no-pmc > gpurun_out/r5_mesh50k_$v.json 2>> gpurun_out/r5_mesh50k_ab.err || exit $?
  echo "$v $(python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"])' gpurun_out/r5_mesh50k_$v.json)" >> gpurun_out/r5_mesh50k_ab.log
done
