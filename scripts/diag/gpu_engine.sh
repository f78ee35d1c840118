#!/bin/bash
# Native engine (libmft) on the GPU: small eager run, then graph-captured headline-shape run.
set -o pipefail
mkdir -p gpurun_out
B=mobilefinetuner_amd/bin/gpt2_lora_finetune
timeout -k 10 120 $B --random_init --model gpt2-tiny --synthetic_data --synthetic_tokens 200000 --steps 6 \
  --batch_size 4 --seq_len 64 --lr 1e-3 --no_graph > gpurun_out/eng_tiny_eager.log 2>&1
rc=$?; tail -12 gpurun_out/eng_tiny_eager.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 $B --random_init --model gpt2-tiny --synthetic_data --synthetic_tokens 200000 --steps 6 \
  --batch_size 4 --seq_len 64 --lr 1e-3 > gpurun_out/eng_tiny_graph.log 2>&1
rc=$?; tail -8 gpurun_out/eng_tiny_graph.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 $B --random_init --model gpt2 --synthetic_data --synthetic_tokens 3000000 --steps 30 \
  --batch_size 512 --seq_len 128 --lr 1e-4 --log_interval 10 > gpurun_out/eng_gpt2.log 2>&1
rc=$?; tail -12 gpurun_out/eng_gpt2.log; exit $rc
