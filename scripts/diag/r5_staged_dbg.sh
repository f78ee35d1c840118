#!/bin/bash
# staged ZeRO-3 optimizer: one loopback rank in graph mode with the streamed-optimizer trace
set -o pipefail
O=gpurun_out/r5sdbg
mkdir -p $O
A="--random_init --model gpt2-tiny --synthetic_data --synthetic_tokens 100000 --seq_len 64 --lr 1e-3 --log_interval 1 --deterministic --steps 4 --bucket_mb 0.25 --batch_size 4 --zero_stage 3 --offload host --offload_moments fp32"
MFT_DP_FORCE_COMM=1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29611 MFT_COMM_BACKEND=loopback MFT_Z3_TRACE=1 timeout -k 10 120 mobilefinetuner_amd/bin/gpt2_full_finetune $A > $O/run.txt 2>&1; rc=$?
echo "rc=$rc"; tail -40 $O/run.txt | cut -c1-200
