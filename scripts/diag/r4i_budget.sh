#!/bin/bash
# CE E-buffer budget default A/B: 4 GiB vs 6.5 GiB on the headline and Gemma-3, interleaved rounds
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r4i_budget.txt
for r in 1 2 3; do
  for b in 4 6.5; do
    for c in gpt2-lora gemma3-270m-lora; do
      MFT_CE_BUDGET_GB=$b timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 5 > gpurun_out/r4i_one.txt 2>&1 || { tail -5 gpurun_out/r4i_one.txt; exit 1; }
      echo "round $r budget $b $c $(tail -1 gpurun_out/r4i_one.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), d["ms_per_step"], d["config"].get("peak_hbm_gb_rank0"))')" | tee -a gpurun_out/r4i_budget.txt
    done
  done
done
