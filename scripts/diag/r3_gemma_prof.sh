#!/bin/bash
# native Gemma-3 step profile, eager (rocprofv3 --kernel-trace segfaults inside hipGraphLaunch of the Gemma
# step graph -- the same binary runs clean without the profiler -- so the kernels are traced un-captured)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
ARGS="--model gemma3-270m --random_init --synthetic_data --synthetic_tokens 2000000 --batch 256 --seq_len 256 --lora_dropout 0 --targets full"
rm -rf gpurun_out/p_gemma
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p_gemma -o run -- mobilefinetuner_amd/bin/train_lora_gemma $ARGS --max_steps 15 --log_interval 0 --bench_steps 10 --bench_warmup 5 --no_graph > gpurun_out/r3g_prof.log 2>&1; rc=$?
echo "prof bench-mode rc=$rc"; grep MFT_BENCH gpurun_out/r3g_prof.log | cut -c1-150
[ $rc -eq 0 ] || { grep -v "^\s*@" gpurun_out/r3g_prof.log | tail -5; exit 1; }
DB=$(find gpurun_out/p_gemma -name "*.db" | head -1)
python3 scripts/prof_db.py $DB stats 15 40 > gpurun_out/r3_native_gemma_kernel_stats.txt
rm -rf gpurun_out/p_gemma
head -30 gpurun_out/r3_native_gemma_kernel_stats.txt | cut -c1-160
rm -rf gpurun_out/p_gpt2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p_gpt2 -o run -- mobilefinetuner_amd/bin/gpt2_lora_finetune --random_init --synthetic_data --synthetic_tokens 2000000 --batch_size 1024 --seq_len 128 --steps 15 --log_interval 0 --bench_steps 10 --bench_warmup 5 > gpurun_out/r3p_gpt2.log 2>&1 || { tail -5 gpurun_out/r3p_gpt2.log; exit 1; }
DB=$(find gpurun_out/p_gpt2 -name "*.db" | head -1)
python3 scripts/prof_db.py $DB stats 15 40 > gpurun_out/r3_native_gpt2_kernel_stats.txt
rm -rf gpurun_out/p_gpt2
head -24 gpurun_out/r3_native_gpt2_kernel_stats.txt | cut -c1-160
