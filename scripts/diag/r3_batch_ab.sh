#!/bin/bash
# headline micro-batch A/B: GPT-2 LoRA 1024 vs 2048 x 128, Gemma-3 LoRA 256 vs 512 x 256 (interleaved)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
rm -f gpurun_out/r3_batch_ab.txt
for r in 1 2; do
  for v in "gpt2-lora 1024" "gpt2-lora 2048" "gemma3-270m-lora 256" "gemma3-270m-lora 512"; do
    set -- $v
    timeout -k 10 300 python3 bench.py --config $1 --batch $2 --steps 20 --warmup 5 > gpurun_out/r3_b_one.json 2> gpurun_out/r3_b.err || { tail -20 gpurun_out/r3_b.err; exit 1; }
    echo "$1 batch $2: $(python3 -c 'import json; r=json.load(open("gpurun_out/r3_b_one.json")); print(r["value"], r["ms_per_step"], r["config"]["peak_hbm_gb_rank0"])')" | tee -a gpurun_out/r3_batch_ab.txt
  done
done
