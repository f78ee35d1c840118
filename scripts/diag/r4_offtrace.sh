#!/bin/bash
# kernel timeline of the streamed ZeRO-3 offload step (GPT-2 XL): do the per-unit AdamW updates overlap the forward?
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
B=$PWD/mobilefinetuner_amd/bin/gpt2_full_finetune
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d $PWD/gpurun_out/r4_offtrace -o run -- $B --random_init --model gpt2-xl --synthetic_data --synthetic_tokens 2000000 --seq_len 128 --batch_size 256 --steps 5 --log_interval 1 --lr 1e-5 --zero_stage 3 --offload host > gpurun_out/r4_offtrace.log 2>&1 || { tail -20 gpurun_out/r4_offtrace.log; exit 1; }
grep "Train\]" gpurun_out/r4_offtrace.log | tail -3
F=$(find gpurun_out/r4_offtrace -name "*kernel_trace.csv" | head -1)
H=$(find gpurun_out/r4_offtrace -name "*hip_api_trace.csv" | head -1)
python3 scripts/diag/r4_offtrace.py $F cols $H > gpurun_out/r4_offtrace_summary.txt; cat gpurun_out/r4_offtrace_summary.txt
rm -f $F $H
