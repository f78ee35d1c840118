#!/bin/bash
# full fine-tune micro-batch A/B: GPT-2 XL ZeRO-3 64 / 128 / 256 x 128, GPT-2 full 512 / 1024 x 128
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
rm -f gpurun_out/r3_fullbatch_ab.txt
for v in "gpt2-xl-zero3 64" "gpt2-xl-zero3 128" "gpt2-xl-zero3 256" "gpt2-full 512" "gpt2-full 1024" "gpt2-xl-zero3 64" "gpt2-xl-zero3 256" "gpt2-xl-zero3-offload 64" "gpt2-xl-zero3-offload 256"; do
  set -- $v
  timeout -k 10 400 python3 bench.py --config $1 --batch $2 --steps 10 --warmup 3 > gpurun_out/r3_fb_one.json 2> gpurun_out/r3_fb.err || { tail -20 gpurun_out/r3_fb.err; exit 1; }
  echo "$1 batch $2: $(python3 -c 'import json; r=json.load(open("gpurun_out/r3_fb_one.json")); print(r["value"], r["ms_per_step"], r["config"]["peak_hbm_gb_rank0"], r["config"]["mfu_bf16_dense"])')" | tee -a gpurun_out/r3_fullbatch_ab.txt
done
