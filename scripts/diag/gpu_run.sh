#!/bin/bash
# Run GPU steps in sequence; stop at the first step that crashes / times out (exit not 0/1).
# usage: scripts/gpu_run.sh "<timeout_s>::<name>::<cmd>" ...
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for spec in "$@"; do
  t="${spec%%::*}"; rest="${spec#*::}"; name="${rest%%::*}"; cmd="${rest#*::}"
  echo "=== [$name] $cmd (timeout ${t}s)"
  start=$(date +%s)
  timeout -k 10 "$t" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "=== stopping: step $name ended with rc=$rc"
    exit $rc
  fi
done
exit 0
