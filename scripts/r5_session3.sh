#!/bin/bash
# Round-5 GPU session 3 (DEV TOOL): tests + smoke, then triangle leaf sizes on mesh50k
bash scripts/gpu_tests.sh r5c; rc=$?
echo "tests rc=$rc" > gpurun_out/r5c_rc.txt
case $rc in 124|134|137|139) exit $rc;; esac
L=gpurun_out/r5_ab_d.log
timeout -k 10 300 bash scripts/ab_lib.sh "mesh50k 128 f64" base tleaf3 tleaf4 > $L 2>&1
r=$?; echo "ab_d rc=$r" >> gpurun_out/r5c_rc.txt; case $r in 124|134|137|139) exit $r;; esac
timeout -k 10 300 bash scripts/ab_lib.sh "mesh50k 128 f64" base tleaf3 tleaf4 >> $L 2>&1
echo "ab_d2 rc=$?" >> gpurun_out/r5c_rc.txt
exit $rc
