#!/bin/bash
# three bench configs (headline, Gemma-3 LoRA, GPT-2 full FT), one JSON line each
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
TAG=${1:-b3}; shift
for c in gpt2-lora gemma3-270m-lora gpt2-full; do
  timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 5 "$@" >> gpurun_out/${TAG}.jsonl 2>> gpurun_out/${TAG}.err || { tail gpurun_out/${TAG}.err; exit 1; }
done
cut -c1-330 gpurun_out/${TAG}.jsonl
