#!/bin/bash
# Arbitrary PMC counter passes (one rocprofv3 run per set) over one probe_speed.py workload.
# usage: bash scripts/pmc_sets.sh <outdir> "<set1>" ["<set2>" ...] -- <probe args...>
# (select a library variant with RT_HIP_LIB in the environment); summarize with scripts/pmc_report.py
out=$1; shift
sets=()
while [ "$1" != "--" ]; do sets+=("$1"); shift; done
shift
cd /tmp && export TMPDIR=/tmp
i=0
for set in "${sets[@]}"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set --output-format csv -d "$out/p$i" -o run -- python3 "$GRAFT_REPO_ROOT/scripts/probe_speed.py" "$@" || exit $?
done
