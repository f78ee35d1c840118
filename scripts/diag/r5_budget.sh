#!/bin/bash
# Gemma-3 CE E-buffer budget A/B: 2 / 4 (default) / 8 GiB, interleaved rounds
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r5_budget.txt
for r in 1 2; do
  for b in 2 4 8; do
    MFT_CE_BUDGET_GB=$b timeout -k 10 300 python3 bench.py --config gemma3-270m-lora --steps 20 --warmup 5 > gpurun_out/r5_one.txt 2>&1 || { tail -5 gpurun_out/r5_one.txt; exit 1; }
    echo "round $r budget $b $(tail -1 gpurun_out/r5_one.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), d["ms_per_step"], d["config"].get("peak_hbm_gb_rank0"))')" | tee -a gpurun_out/r5_budget.txt
  done
done
