#!/bin/bash
# A/B throughput of library variants: usage ab_probe.sh "<config> <spp> <precs> <accel>" variant[:ENV=VAL] ...
args=$1; shift
for spec in "$@"; do
  v=${spec%%:*}; envs=""; [ "$v" != "$spec" ] && envs=${spec#*:}
  echo -n "$spec: "
  env $envs RT_HIP_LIB=blenderraytracer_amd/lib/variants/$v.so timeout -k 10 120 python scripts/probe_speed.py $args 2>&1 | grep Msamples | sed 's/wall.*kernel) //' | tr '\n' ' ' || exit 1
  echo
done
