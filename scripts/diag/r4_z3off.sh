#!/bin/bash
# ZeRO-3 host-streamed optimizer under graph capture: single process, with trace lines + backtraces
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
B=mobilefinetuner_amd/bin/gpt2_full_finetune
ARGS="--random_init --model gpt2-tiny --synthetic_data --synthetic_tokens 100000 --seq_len 64 --lr 1e-3 --log_interval 1 --deterministic --steps 6 --batch_size 4 --zero_stage 3 --offload host"
MFT_Z3_TRACE=1 MFT_DP_FORCE_COMM=1 MFT_COMM_BACKEND=loopback RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29611 \
  timeout -k 10 120 $B $ARGS > gpurun_out/r4_z3off_1.log 2>&1; rc=$?; echo "1-rank graph rc=$rc"
tail -22 gpurun_out/r4_z3off_1.log
exit 0
