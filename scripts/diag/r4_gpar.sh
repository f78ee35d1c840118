#!/bin/bash
# graph branch concurrency under the runtime's graph settings
set -o pipefail
mkdir -p gpurun_out
P=scripts/diag/r4_graph_par
O=gpurun_out/r4_graph_par.txt; : > $O
for e in "X=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "DEBUG_HIP_FORCE_GRAPH_QUEUES=2" "DEBUG_HIP_FORCE_GRAPH_QUEUES=4" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 DEBUG_HIP_FORCE_GRAPH_QUEUES=4"; do
  echo "== $e" | tee -a $O
  env $e timeout -k 10 60 $P >> $O 2>&1 || { echo "rc=$?" | tee -a $O; exit 1; }
done
cat $O
