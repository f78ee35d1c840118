#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-r5b4}
mkdir -p $O
export TMPDIR=/tmp
B="--random_init --synthetic_data --synthetic_tokens 2000000 --seq_len 128 --batch_size 4 --steps 70 --log_interval 0 --bench_steps 50 --bench_warmup 10 --no_graph"
rm -rf $O/p
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p -o run -- mobilefinetuner_amd/bin/gpt2_lora_finetune $B > $O/b4.log 2>&1 || { tail -5 $O/b4.log; exit 1; }
DB=$(find $O/p -name "*.db" | head -1)
python3 scripts/prof_db.py $DB stats 70 70 > $O/b4_kernel_stats.txt && head -60 $O/b4_kernel_stats.txt | cut -c1-150
python3 scripts/prof_db.py $DB step > $O/b4_step.txt 2>&1; tail -5 $O/b4_step.txt | cut -c1-150
rm -rf $O/p
