#!/bin/bash
# native weight streaming A/B: HBM peak and throughput, resident vs --shard_enable
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B=mobilefinetuner_amd/bin
run() {  # tag, cmd...
  local tag=$1; shift
  timeout -k 10 300 "$@" > gpurun_out/ws_$tag.log 2>&1 || { tail -5 gpurun_out/ws_$tag.log; return 1; }
  echo "$tag: $(grep -E 'weight streaming ON' gpurun_out/ws_$tag.log | head -1)"
  echo "   $(grep -E 'tokens/s\)|HBM' gpurun_out/ws_$tag.log | tail -2 | tr '\n' ' ')"
}
G="--random_init --synthetic_data --synthetic_tokens 2000000 --steps 30 --batch_size 16 --seq_len 128 --log_interval 10"
run gpt2_resident $B/gpt2_lora_finetune --model gpt2-medium $G && \
run gpt2_stream $B/gpt2_lora_finetune --model gpt2-medium $G --shard_enable --shard_budget_mb 128 && \
M="--random_init --model gemma3-1b --synthetic_data --synthetic_tokens 2000000 --max_steps 20 --batch 8 --seq_len 256 --log_interval 10 --eval_batches 1"
run gemma_resident $B/train_lora_gemma $M && \
run gemma_stream $B/train_lora_gemma $M --shard_enable --shard_budget_mb 256
