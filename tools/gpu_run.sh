#!/bin/bash
# Run GPU steps in order; stop at the first crash/abort/timeout (exit 124, 134,
# 137, 139 or negative-signal codes) so no further GPU work starts after a fault.
# Usage: tools/gpu_run.sh "<name>:<seconds>:<command>" ...
mkdir -p gpurun_out
for step in "$@"; do
  name="${step%%:*}"; rest="${step#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== $name ($secs s): $cmd"
  mkdir -p "$(dirname "gpurun_out/$name.log")"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc"
  tail -n 15 "gpurun_out/$name.log"
  case $rc in
    0|1|2|5) ;;                        # pass / test failures: keep going
    *) echo "=== stopping after $name (rc=$rc)"; exit $rc ;;
  esac
done
