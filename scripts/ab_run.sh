#!/bin/bash
# A/B rounds over library variants (forward then reverse order): usage ab_run.sh "<probe args>" v1 v2 ...
args=$1; shift
V="$*"; R=$(echo $V | tr ' ' '\n' | tac | tr '\n' ' ')
for order in "$V" "$R"; do
  for v in $order; do bash scripts/ab_probe.sh "$args" $v || exit 1; done
done
