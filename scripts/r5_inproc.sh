#!/bin/bash
# Round 5 (DEV TOOL): the one-process multi-device rehearsal (devices [0, 0] on one GPU) — progressive_16
# with one fused launch per device (default) vs one launch per batch (RT_FUSED_BATCHES=0, round 4's
# multi-device form), both orders
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r5_inproc.log
: > $L
for v in fused unfused unfused fused; do
  if [ $v = fused ]; then
    timeout -k 10 300 python3 bench.py --gpus 2 --mp-mode inproc --steps 5 --warmup 1 --no-cpu-baseline --no-pmc > gpurun_out/r5_inproc_$v.json 2>> $L || exit 1
  else
    RT_FUSED_BATCHES=0 timeout -k 10 300 python3 bench.py --gpus 2 --mp-mode inproc --steps 5 --warmup 1 --no-cpu-baseline --no-pmc > gpurun_out/r5_inproc_$v.json 2>> $L || exit 1
  fi
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r5_inproc_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], json.dumps(d.get('progressive_16')))" >> $L
done
