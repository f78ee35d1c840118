#!/bin/bash
# Round 3, first look: native libmft CLIs vs the torch-driven bench path at the headline configs
# (same box), plus a rocprofv3 kernel-stats profile of the native GPT-2 LoRA step.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
B=mobilefinetuner_amd/bin
timeout -k 10 300 $B/gpt2_lora_finetune --random_init --synthetic_data --synthetic_tokens 8000000 \
  --batch_size 1024 --seq_len 128 --steps 30 --log_interval 10 --lr 2e-4 > gpurun_out/r3_nat_gpt2.log 2>&1 \
  || { tail -20 gpurun_out/r3_nat_gpt2.log; exit 1; }
grep -E "Step|tokens/s" gpurun_out/r3_nat_gpt2.log | cut -c1-200
timeout -k 10 300 $B/train_lora_gemma --random_init --synthetic_data --synthetic_tokens 4000000 \
  --batch 256 --seq_len 256 --max_steps 25 --log_interval 5 --lora_dropout 0 --alpha 16 > gpurun_out/r3_nat_gemma.log 2>&1 \
  || { tail -20 gpurun_out/r3_nat_gemma.log; exit 1; }
grep -E "Step|tokens/s" gpurun_out/r3_nat_gemma.log | cut -c1-200
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r3_py_gpt2.json 2>gpurun_out/r3_py_gpt2.err \
  || { tail gpurun_out/r3_py_gpt2.err; exit 1; }
cut -c1-200 gpurun_out/r3_py_gpt2.json
timeout -k 10 300 python3 bench.py --config gemma3-270m-lora --steps 15 --warmup 4 > gpurun_out/r3_py_gemma.json 2>gpurun_out/r3_py_gemma.err \
  || { tail gpurun_out/r3_py_gemma.err; exit 1; }
cut -c1-200 gpurun_out/r3_py_gemma.json
rm -rf gpurun_out/p_nat
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/p_nat -o run -- $B/gpt2_lora_finetune --random_init \
  --synthetic_data --synthetic_tokens 4000000 --batch_size 1024 --seq_len 128 --steps 11 --log_interval 11 \
  > gpurun_out/r3_nat_prof.log 2>&1 || { tail gpurun_out/r3_nat_prof.log; exit 1; }
DB=$(find gpurun_out/p_nat -name "*.db" | head -1)
python3 scripts/prof_db.py $DB stats 11 45 > gpurun_out/r3_nat_gpt2_stats.txt && head -30 gpurun_out/r3_nat_gpt2_stats.txt | cut -c1-160
rm -rf gpurun_out/p_nat
