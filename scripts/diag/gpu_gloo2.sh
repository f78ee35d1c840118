#!/bin/bash
# two ranks on the one GPU over gloo: the bench's multi-rank path (rank spawning, DP reducer after the
# graph replay, ZeRO-2 buckets, rank-max timing) on real hardware
set -o pipefail
export PYTHONPATH=$PWD MFT_DIST_BACKEND=gloo
mkdir -p gpurun_out
: > gpurun_out/gloo2.jsonl
for args in "--config gpt2-lora" "--config gpt2-full" "--config gpt2-full --zero 2"; do
  echo "bench --gpus 2 $args"
  timeout -k 10 400 python bench.py --gpus 2 $args --steps 6 --warmup 3 >> gpurun_out/gloo2.jsonl 2> gpurun_out/gloo2.err || { tail -30 gpurun_out/gloo2.err; exit 1; }
done
cut -c1-330 gpurun_out/gloo2.jsonl
