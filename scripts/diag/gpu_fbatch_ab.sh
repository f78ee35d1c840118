#!/bin/bash
# GPT-2 full fine-tune micro-batch A/B (sequences per GPU per step), interleaved
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
: > gpurun_out/fbatch_ab.txt
for r in 1 2; do
  for b in 512 1024; do
    out=$(timeout -k 10 300 python3 bench.py --config gpt2-full --batch $b --steps 20 --warmup 5 2> gpurun_out/fbatch_ab.err) || { tail -5 gpurun_out/fbatch_ab.err; exit 1; }
    echo "batch=$b $(echo "$out" | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" | tee -a gpurun_out/fbatch_ab.txt
  done
done
