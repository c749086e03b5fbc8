#!/bin/bash
# GPU tests + smoke, then an A/B script, in one box session (DEV TOOL).  A failing test does not stop
# the A/B; a fault, abort or time limit (status 124, 134, 137, 139) ends the session there.
# usage: bash scripts/gpu_round.sh <tag> [ab script]
tag=$1; ab=$2
bash scripts/gpu_tests.sh $tag; rc=$?
echo "tests rc=$rc" > gpurun_out/${tag}_rc.txt
case $rc in 124|134|137|139) exit $rc;; esac
[ -n "$ab" ] && { timeout -k 10 700 bash $ab; echo "ab rc=$?" >> gpurun_out/${tag}_rc.txt; }
exit $rc
