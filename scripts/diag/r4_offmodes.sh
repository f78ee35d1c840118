#!/bin/bash
# ZeRO-3 host-offloaded AdamW on GPT-2 XL: per-unit streamed (in place, during the next forward) vs one
# in-place update after the backward; bf16 and fp32 moments
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/r4_offload_modes.txt; : > $O
for m in stream zerocopy; do
  for f in "" --offload_fp32; do
    timeout -k 10 300 python3 bench.py --config gpt2-xl-zero3-offload --offload_mode $m $f --steps 10 --warmup 3 > gpurun_out/r4_om.txt 2>&1 || { tail -5 gpurun_out/r4_om.txt; exit 1; }
    echo "mode=$m ${f:-bf16} $(tail -1 gpurun_out/r4_om.txt | cut -c1-330)" | tee -a $O
  done
done
