#!/bin/bash
# Round-6 GPU session 1 (DEV TOOL): the GPU tier with the new queue / gamma / resume tests, smoke, and
# baseline probes of configs 3 and 5 for the round's A/B runs
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r6a_tests.log 2>&1
rc=$?; echo "tests rc=$rc" > gpurun_out/r6a_rc.txt
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6a_smoke.log 2>&1
r=$?; echo "smoke rc=$r" >> gpurun_out/r6a_rc.txt; case $r in 124|134|137|139) exit $r;; esac
for w in "rtow 256 f64" "mesh50k 128 f64" "rtow 256 f64" "mesh50k 128 f64"; do
  timeout -k 10 120 python scripts/probe_speed.py $w >> gpurun_out/r6a_probe.log 2>&1 || exit $?
done
exit $rc
