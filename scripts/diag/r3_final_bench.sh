#!/bin/bash
# round-3 closing run, part 2: every bench config on one GPU + a kernel profile of the headline step
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
rm -f gpurun_out/r3_final_bench.jsonl
for cfg in gpt2-lora gemma3-270m-lora gpt2-full gpt2-xl-zero gpt2-xl-zero3 gpt2-xl-zero3-offload; do
  timeout -k 10 600 python3 bench.py --config $cfg --steps 20 --warmup 5 >> gpurun_out/r3_final_bench.jsonl 2> gpurun_out/r3_final_$cfg.err || { tail -20 gpurun_out/r3_final_$cfg.err; exit 1; }
  echo "$cfg: $(tail -1 gpurun_out/r3_final_bench.jsonl | cut -c1-200)"
done
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 >> gpurun_out/r3_final_bench.jsonl 2>> gpurun_out/r3_final_gpt2-lora.err && echo "gpt2-lora (2nd): $(tail -1 gpurun_out/r3_final_bench.jsonl | cut -c1-160)"
rm -rf gpurun_out/p_final
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p_final -o run -- mobilefinetuner_amd/bin/gpt2_lora_finetune \
  --random_init --synthetic_data --synthetic_tokens 2000000 --batch_size 1024 --seq_len 128 --steps 15 --log_interval 0 --bench_steps 10 --bench_warmup 5 > gpurun_out/r3_final_prof.log 2>&1 || { tail gpurun_out/r3_final_prof.log; exit 1; }
DB=$(find gpurun_out/p_final -name "*.db" | head -1)
python3 scripts/prof_db.py $DB stats 15 40 > gpurun_out/r3_final_gpt2_lora_stats.txt
rm -rf gpurun_out/p_final
head -14 gpurun_out/r3_final_gpt2_lora_stats.txt
