#!/bin/bash
# Round-5 GPU session 2 (DEV TOOL): tests + smoke, the Node host test with its prints, the fused-batch
# stress (single and multi-device), then A/B set c
bash scripts/gpu_tests.sh r5b; rc=$?
echo "tests rc=$rc" > gpurun_out/r5b_rc.txt
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python -u -m pytest tests/test_js_host.py -x -q -s -m gpu -k "matches_reference" > gpurun_out/r5b_js.log 2>&1
r=$?; echo "js rc=$r" >> gpurun_out/r5b_rc.txt; case $r in 124|134|137|139) exit $r;; esac
timeout -k 10 500 python -u scripts/stress_fused.py 150 > gpurun_out/r5b_stress.log 2>&1
r=$?; echo "stress rc=$r" >> gpurun_out/r5b_rc.txt; case $r in 124|134|137|139) exit $r;; esac
timeout -k 10 700 bash scripts/ab_r5c.sh; echo "ab_c rc=$?" >> gpurun_out/r5b_rc.txt
exit $rc
