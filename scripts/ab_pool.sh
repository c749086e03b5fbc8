#!/bin/bash
# A/B of the sample pool against the lane-per-pixel kernel and of pool chunk sizes (full-spp probes)
# usage: bash scripts/ab_pool.sh "<config> <spp> <prec>" "label:ENV=V ENV2=V" ...
args=$1; shift
for r in 1 2; do
  for spec in "$@"; do
    label=${spec%%:*}; envs=${spec#*:}
    echo -n "$label: "; env $envs timeout -k 10 120 python scripts/probe_speed.py $args 2>&1 | grep Msamples || exit 1
  done
done
