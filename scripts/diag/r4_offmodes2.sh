#!/bin/bash
# streamed in-place ZeRO-3 offload: optimizer grid size / stream priority sweep (bf16 moments)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/r4_offload_modes2.txt; : > $O
for cfg in "256 1" "64 1" "1024 1" "256 0" "2048 0"; do
  set -- $cfg
  MFT_Z3_OPT_GRID=$1 MFT_Z3_OPT_PRIO=$2 timeout -k 10 300 python3 bench.py --config gpt2-xl-zero3-offload --offload_mode stream --steps 10 --warmup 3 > gpurun_out/r4_om.txt 2>&1 || { tail -5 gpurun_out/r4_om.txt; exit 1; }
  echo "grid=$1 lowprio=$2 $(tail -1 gpurun_out/r4_om.txt | cut -c1-250)" | tee -a $O
done
