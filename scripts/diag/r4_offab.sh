#!/bin/bash
# streamed ZeRO-3 offload (in place, 4 float4 groups in flight per thread): optimizer grid sweep vs zerocopy
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
B=mobilefinetuner_amd/bin/gpt2_full_finetune
A="--random_init --model gpt2-xl --synthetic_data --synthetic_tokens 2000000 --seq_len 128 --batch_size 256 --steps 6 --log_interval 1 --lr 1e-5 --zero_stage 3 --offload host"
O=gpurun_out/r4_offab3.txt; : > $O
run() {  # label, env...
  local label=$1; shift
  env "$@" timeout -k 10 240 $B $A $EXTRA > gpurun_out/r4_offab_run.log 2>&1 || { tail -5 gpurun_out/r4_offab_run.log; exit 1; }
  echo "$label: $(grep 'Train\]' gpurun_out/r4_offab_run.log | tail -3 | sed 's/.*step_ms/step_ms/' | tr '\n' ' ')" | tee -a $O
}
for g in 24 32 48; do EXTRA="" run "stream grid=$g U=8" MFT_Z3_OPT_GRID=$g MFT_OPT_UNROLL=8; done
EXTRA="" run "stream grid=32 U=4" MFT_Z3_OPT_GRID=32
EXTRA="--offload_moments fp32" run "stream fp32 grid=32 U=8" MFT_Z3_OPT_GRID=32 MFT_OPT_UNROLL=8
EXTRA="--offload_moments fp32" run "stream fp32 grid=48 U=4" MFT_Z3_OPT_GRID=48
