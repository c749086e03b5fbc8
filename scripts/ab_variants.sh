#!/bin/bash
# A/B: f64 RTOW throughput per library variant (probe at reduced spp); args: variant[:path] ...
for spec in "$@"; do
  v=${spec%%:*}; p=${spec#*:}; [ "$p" = "$spec" ] && p=smem
  echo -n "$v $p: "
  RT_HIP_LIB=blenderraytracer_amd/lib/variants/$v.so RT_SPHERE_PATH=$p timeout -k 10 120 python scripts/probe_speed.py rtow 64 f64 2>&1 | grep Msamples || exit 1
done
