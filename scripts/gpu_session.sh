#!/bin/bash
# One gpurun session: each GPU step under its own timeout; stop at the first crash/timeout/abort.
# usage: bash scripts/gpu_session.sh "<label>:<seconds>:<command>" ...
mkdir -p gpurun_out
for spec in "$@"; do
  label="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$label] ($secs s) $cmd" | tee -a gpurun_out/session.log
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$label.log" 2>&1
  rc=$?
  echo "=== [$label] exit $rc" | tee -a gpurun_out/session.log
  tail -5 "gpurun_out/$label.log"
  # 0 ok, 1 test failures / python error: keep going; anything else (124/137 timeout, 134 abort,
  # 139 segv, ...) may mean a sick GPU: stop here
  if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 2 ]; then echo "stopping after [$label] rc=$rc"; exit $rc; fi
done
