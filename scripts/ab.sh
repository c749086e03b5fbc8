#!/bin/bash
# Interleaved A/B of library variants and environment switches on one probe workload (DEV TOOL).
# usage: bash scripts/ab.sh [-r REPS] "<config> <spp> <prec>" SPEC...
#   SPEC = name:SETTINGS, SETTINGS a comma list of VAR=value (environment) and @variant (a library built
#   by scripts/build_variants.sh); "name:" alone is the default build and environment.
#   e.g. bash scripts/ab.sh -r 2 "mesh50k 128 f64" base: tri_lds:RT_LDS_TRI=1 w8:@w8,RT_LDS_TRI=1
# Every repetition runs the specs in order, then in reverse order (drift cancels); each line is
# probe_speed.py's Msamples/s line prefixed with the spec's name.
reps=1
if [ "$1" = "-r" ]; then reps=$2; shift 2; fi
args=$1; shift
specs=("$@")
run_spec() {
  local name=${1%%:*} settings=${1#*:} envs=() lib=""
  IFS=',' read -ra parts <<< "$settings"
  for p in "${parts[@]}"; do
    case $p in
      @*) lib="blenderraytracer_amd/lib/variants/${p#@}.so" ;;
      *=*) envs+=("$p") ;;
    esac
  done
  [ -n "$lib" ] && envs+=("RT_HIP_LIB=$lib")
  echo -n "$name: "
  env "${envs[@]}" timeout -k 10 120 python scripts/probe_speed.py $args 2>&1 | grep Msamples || return 1
}
for ((r = 0; r < reps; ++r)); do
  for ((i = 0; i < ${#specs[@]}; ++i)); do run_spec "${specs[$i]}" || exit 1; done
  for ((i = ${#specs[@]} - 1; i >= 0; --i)); do run_spec "${specs[$i]}" || exit 1; done
done
