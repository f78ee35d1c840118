#!/bin/bash
# kernel tables: gpt2-lora (graph), gemma3-270m-lora (graph), the reference recipe 4 x 128 (eager, kernel count)
set -o pipefail
O=gpurun_out/${1:-r5prof}
mkdir -p $O
export TMPDIR=/tmp
A="--random_init --synthetic_data --synthetic_tokens 2000000 --seq_len 128 --batch_size 1024 --steps 14 --log_interval 0 --bench_steps 6 --bench_warmup 4"
rm -rf $O/p
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p -o run -- mobilefinetuner_amd/bin/gpt2_lora_finetune $A > $O/g2.log 2>&1 || { tail -5 $O/g2.log; exit 1; }
python3 scripts/prof_db.py $(find $O/p -name "*.db" | head -1) stats 10 40 > $O/gpt2_lora_kernel_stats.txt && head -30 $O/gpt2_lora_kernel_stats.txt | cut -c1-150
rm -rf $O/p
G="--model gemma3-270m --random_init --synthetic_data --synthetic_tokens 2000000 --batch 256 --seq_len 256 --lora_dropout 0 --targets full --max_steps 12 --log_interval 0 --bench_steps 6 --bench_warmup 4"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p -o run -- mobilefinetuner_amd/bin/train_lora_gemma $G > $O/gm.log 2>&1 || { tail -5 $O/gm.log; exit 1; }
python3 scripts/prof_db.py $(find $O/p -name "*.db" | head -1) stats 10 40 > $O/gemma_kernel_stats.txt && head -30 $O/gemma_kernel_stats.txt | cut -c1-150
rm -rf $O/p
B="--random_init --synthetic_data --synthetic_tokens 2000000 --seq_len 128 --batch_size 4 --steps 70 --log_interval 0 --bench_steps 50 --bench_warmup 10 --no_graph"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p -o run -- mobilefinetuner_amd/bin/gpt2_lora_finetune $B > $O/b4.log 2>&1 || { tail -5 $O/b4.log; exit 1; }
python3 scripts/prof_db.py $(find $O/p -name "*.db" | head -1) stats 70 60 > $O/b4_kernel_stats.txt && head -45 $O/b4_kernel_stats.txt | cut -c1-150
rm -rf $O/p
