#!/bin/bash
# lora_rowdot load batch 4 (default) vs 8 (MFT_ROWDOT_UNR=8): micro-bench at the GPT-2 / Gemma shapes
set -o pipefail
O=gpurun_out/r5rowdot
mkdir -p $O
export PYTHONPATH=.
for u in 4 8 4 8; do
  MFT_ROWDOT_UNR=$u timeout -k 10 200 python3 scripts/bench_lora_kernels.py --M 131072 --iters 50 > $O/u$u.txt 2>&1 || { tail -5 $O/u$u.txt; exit 1; }
  echo "UNR=$u"; grep rowdot $O/u$u.txt | grep "p=0" | head -4
done
