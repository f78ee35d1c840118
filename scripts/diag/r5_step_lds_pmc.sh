#!/bin/bash
# LDS bank-conflict counters for every kernel of the gpt2-lora and gemma3 steps (eager, a few steps)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5steppmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
A="--random_init --synthetic_data --synthetic_tokens 2000000 --seq_len 128 --batch_size 1024 --steps 3 --log_interval 0 --no_graph"
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES -d $O/g2 -o run -- $R/mobilefinetuner_amd/bin/gpt2_lora_finetune $A > $O/g2.log 2>&1 || { tail -5 $O/g2.log; exit 1; }
G="--model gemma3-270m --random_init --synthetic_data --synthetic_tokens 2000000 --batch 256 --seq_len 256 --lora_dropout 0 --targets full --max_steps 3 --log_interval 0 --no_graph"
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES -d $O/gm -o run -- $R/mobilefinetuner_amd/bin/train_lora_gemma $G > $O/gm.log 2>&1 || { tail -5 $O/gm.log; exit 1; }
cd $R
python3 scripts/pmc_db.py $(find $O/g2 -name "*.db" | head -1) > $O/g2.txt 2>&1
python3 scripts/pmc_db.py $(find $O/gm -name "*.db" | head -1) > $O/gm.txt 2>&1
rm -rf $O/g2 $O/gm
wc -l $O/g2.txt $O/gm.txt
