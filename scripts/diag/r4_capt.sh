#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
P=scripts/diag/r4_capture_probe
for v in 10 7; do
  timeout -k 10 60 $P $v > gpurun_out/r4_capt_$v.log 2>&1; rc=$?
  echo "variant $v rc=$rc"; cat gpurun_out/r4_capt_$v.log
  [ $rc -ne 0 ] && break
done
exit 0
