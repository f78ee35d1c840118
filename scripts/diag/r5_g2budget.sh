#!/bin/bash
# GPT-2 LoRA headline: CE E-buffer budget A/B (4 GiB default = 4 row chunks; 8 = 2; 16 = 1 chunk), interleaved
set -o pipefail
O=gpurun_out/r5g2b
mkdir -p $O
for r in 1 2; do
  for b in 4 16 8; do
    MFT_CE_BUDGET_GB=$b timeout -k 10 300 python3 bench.py --config gpt2-lora --steps 20 --warmup 5 > $O/one.txt 2>&1 || { tail -5 $O/one.txt; exit 1; }
    echo "round $r budget $b $(tail -1 $O/one.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), d["ms_per_step"], d["config"].get("peak_hbm_gb_rank0"))')"
  done
done
