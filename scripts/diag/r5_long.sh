#!/bin/bash
# longer native training runs on the final kernels: finite, decreasing losses (synthetic data, random init)
set -o pipefail
O=gpurun_out/r5long
mkdir -p $O
A="--random_init --synthetic_data --synthetic_tokens 4000000 --seq_len 128 --batch_size 64 --steps 300 --log_interval 50 --lr 3e-4"
timeout -k 10 300 mobilefinetuner_amd/bin/gpt2_lora_finetune $A > $O/g2.txt 2>&1 || { tail -5 $O/g2.txt; exit 1; }
grep "\[Train\]" $O/g2.txt | cut -c1-150 | tail -7
G="--model gemma3-270m --random_init --synthetic_data --synthetic_tokens 4000000 --batch 16 --seq_len 256 --lora_dropout 0 --targets full --max_steps 200 --log_interval 50 --learning_rate 3e-4"
timeout -k 10 300 mobilefinetuner_amd/bin/train_lora_gemma $G > $O/gm.txt 2>&1 || { tail -5 $O/gm.txt; exit 1; }
grep -i "step\|loss" $O/gm.txt | grep -i loss | cut -c1-150 | tail -5
