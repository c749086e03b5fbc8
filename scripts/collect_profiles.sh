#!/bin/bash
# Copy the judged evidence of scripts/profile_round.sh runs from gpurun_out/ into profiles/.
# usage: bash scripts/collect_profiles.sh <round-version prefix, e.g. r02_v1> <tag>...
pre=$1; shift
for t in "$@"; do
  src=gpurun_out/prof_$t
  cp $src/kt/run_kernel_stats.csv profiles/${pre}_${t}_kernel_stats.csv
  grep -E '^"Kind"|trace_pool_(lds_)?kernel|reduce_kernel' $src/kt/run_kernel_trace.csv > profiles/${pre}_${t}_kernel_trace.csv
  tail -1 $src/bench.json > profiles/${pre}_${t}_bench.json
  for p in fetch write sq vmem; do
    f=$(find $src/pmc/$p -name '*counter_collection.csv' | head -1)
    [ -n "$f" ] && cp "$f" profiles/${pre}_${t}_pmc_${p}.csv
  done
done
ls profiles | grep "^$pre" | wc -l
