#!/bin/bash
# A/B of library variants (scripts/build_variants.sh) on one probe workload, both orders
# usage: bash scripts/ab_lib.sh "<config> <spp> <prec>" variant ...
args=$1; shift
V="$*"; R=$(echo $V | tr ' ' '\n' | tac | tr '\n' ' ')
for order in "$V" "$R"; do
  for v in $order; do
    echo -n "$v: "; RT_HIP_LIB=blenderraytracer_amd/lib/variants/$v.so timeout -k 10 120 python scripts/probe_speed.py $args 2>&1 | grep Msamples || exit 1
  done
done
