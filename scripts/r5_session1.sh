#!/bin/bash
# Round-5 GPU session 1 (DEV TOOL): tests + smoke, then A/B sets a and b
bash scripts/gpu_round.sh r5a scripts/ab_r5a.sh; rc=$?
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 600 bash scripts/ab_r5b.sh; echo "ab_b rc=$?" >> gpurun_out/r5a_rc.txt
exit $rc
