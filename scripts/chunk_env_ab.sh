#!/bin/bash
# pool chunk A/B through RT_POOL_CHUNK on one probe workload, both orders (DEV TOOL)
# usage: bash scripts/chunk_env_ab.sh "<config> <spp> <prec>" chunk ...   (0 = the library's rule)
args=$1; shift
V="$*"; R=$(echo $V | tr ' ' '\n' | tac | tr '\n' ' ')
for order in "$V" "$R"; do
  for c in $order; do
    echo -n "chunk $c: "
    if [ "$c" = 0 ]; then timeout -k 10 120 python scripts/probe_speed.py $args | grep Msamples || exit 1
    else RT_POOL_CHUNK=$c timeout -k 10 120 python scripts/probe_speed.py $args | grep Msamples || exit 1; fi
  done
done
