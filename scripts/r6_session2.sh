#!/bin/bash
# Round-6 GPU session 2 (DEV TOOL): triangle-tree LDS kernel (ACC_BVH_TRI_LDS) parity + A/B against the
# one-wave kernel on mesh50k; the queue-ownership test at 4K
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  -k "mesh50k or cfg5 or queues or triangle or sample_mesh or kitchen" > gpurun_out/r6b_tests.log 2>&1
rc=$?; echo "tests rc=$rc" > gpurun_out/r6b_rc.txt
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 400 bash scripts/ab.sh "mesh50k 128 f64" onewave:RT_LDS_TRI=0 lds: lds255:RT_TRI_LDS_NODES=255 lds64:RT_TRI_LDS_NODES=64 w8:@w8 > gpurun_out/r6b_ab.log 2>&1
r=$?; echo "ab rc=$r" >> gpurun_out/r6b_rc.txt
exit $rc
