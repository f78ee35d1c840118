#!/bin/bash
# Gemma-3 LoRA micro-batch A/B (sequences per GPU per step), interleaved
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
: > gpurun_out/gbatch_ab.txt
for r in 1 2; do
  for b in 256 512; do
    out=$(timeout -k 10 300 python3 bench.py --config gemma3-270m-lora --batch $b --steps 20 --warmup 5 2> gpurun_out/gbatch_ab.err) || { tail -5 gpurun_out/gbatch_ab.err; exit 1; }
    echo "batch=$b $(echo "$out" | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" | tee -a gpurun_out/gbatch_ab.txt
  done
done
