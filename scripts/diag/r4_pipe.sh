#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r4_pipe_probe.txt; : > $O
for a in "1 64" "2 64" "3 64" "1 1024" "3 1024"; do
  timeout -k 10 60 scripts/diag/r4_pipe_probe $a >> $O 2>&1 || { echo "rc=$?" >> $O; cat $O; exit 1; }
done
cat $O
