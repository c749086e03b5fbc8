#!/bin/bash
# Round-4 A/B set (DEV TOOL): grid density and pool chunk under the round-4 kernel (RTOW f64), and
# the top-levels-first node layout on mesh50k.  -> gpurun_out/r4_ab_b.log
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r4_ab_b.log
echo "-- grid density (cells per sphere)" > $L
timeout -k 10 200 bash scripts/ab_lib.sh "rtow 256 f64" cur lam0125 lam018 lam035 >> $L 2>&1 || exit 1
echo "-- pool chunk, RTOW 512 spp" >> $L
for c in 45 32 64 90 45; do echo -n "chunk $c: " >> $L; RT_POOL_CHUNK=$c timeout -k 10 100 python scripts/probe_speed.py rtow 512 f64 2>&1 | grep Msamples >> $L || exit 1; done
echo "-- mesh50k node layout" >> $L
for lay in pre top pre top; do echo -n "$lay: " >> $L; RT_BVH_LAYOUT=$lay timeout -k 10 100 python scripts/probe_speed.py mesh50k 64 f64 2>&1 | grep Msamples >> $L || exit 1; done
echo "-- grid from global memory (RT_LDS_GRID=0): survivor masks there too (gcomp) vs before (cur)" >> $L
RT_LDS_GRID=0 timeout -k 10 120 bash scripts/ab_lib.sh "rtow 128 f64" cur gcomp >> $L 2>&1 || exit 1
echo "-- RT_PROFILE split (RTOW 256 spp f64)" >> $L
RT_HIP_LIB=blenderraytracer_amd/lib/variants/prof.so timeout -k 10 100 python scripts/probe_speed.py rtow 256 f64 >> $L 2>&1 || exit 1
echo "-- filter loop unroll (cur = compiler's choice)" >> $L
timeout -k 10 200 bash scripts/ab_lib.sh "rtow 256 f64" cur fu2 fu4 >> $L 2>&1 || exit 1
