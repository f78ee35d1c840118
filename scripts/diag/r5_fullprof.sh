#!/bin/bash
# kernel table of the gpt2-full bench step (1024 x 128, graph)
set -o pipefail
O=gpurun_out/${1:-r5fullprof}
mkdir -p $O
export TMPDIR=/tmp
A="--random_init --synthetic_data --synthetic_tokens 2000000 --seq_len 128 --batch_size 1024 --steps 14 --log_interval 0 --bench_steps 6 --bench_warmup 4"
rm -rf $O/p
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p -o run -- mobilefinetuner_amd/bin/gpt2_full_finetune $A > $O/full.log 2>&1 || { tail -5 $O/full.log; exit 1; }
python3 scripts/prof_db.py $(find $O/p -name "*.db" | head -1) stats 10 40 > $O/gpt2_full_kernel_stats.txt && head -30 $O/gpt2_full_kernel_stats.txt | cut -c1-170
rm -rf $O/p
