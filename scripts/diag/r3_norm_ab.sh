#!/bin/bash
# norm kernels with the residual-gradient / affine loads hoisted ahead of the row reductions:
# norm + engine tests, Gemma-3 (eager) and GPT-2 step kernel profiles, benches of both LoRA configs
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py > gpurun_out/norm_tests.log 2>&1 || { tail -20 gpurun_out/norm_tests.log; exit 1; }
tail -1 gpurun_out/norm_tests.log
ARGS="--model gemma3-270m --random_init --synthetic_data --synthetic_tokens 2000000 --batch 256 --seq_len 256 --lora_dropout 0 --targets full"
rm -rf gpurun_out/p_gemma
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p_gemma -o run -- mobilefinetuner_amd/bin/train_lora_gemma $ARGS --max_steps 15 --log_interval 0 --bench_steps 10 --bench_warmup 5 --no_graph > gpurun_out/norm_gprof.log 2>&1 || { grep -v "^\s*@" gpurun_out/norm_gprof.log | tail -5; exit 1; }
DB=$(find gpurun_out/p_gemma -name "*.db" | head -1)
python3 scripts/prof_db.py $DB stats 15 40 > gpurun_out/r3_norm_gemma_kernel_stats.txt
rm -rf gpurun_out/p_gemma
grep -E "total|gated|norm_" gpurun_out/r3_norm_gemma_kernel_stats.txt | cut -c1-150
rm -rf gpurun_out/p_gpt2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p_gpt2 -o run -- mobilefinetuner_amd/bin/gpt2_lora_finetune --random_init --synthetic_data --synthetic_tokens 2000000 --batch_size 1024 --seq_len 128 --steps 15 --log_interval 0 --bench_steps 10 --bench_warmup 5 > gpurun_out/norm_pprof.log 2>&1 || { tail -5 gpurun_out/norm_pprof.log; exit 1; }
DB=$(find gpurun_out/p_gpt2 -name "*.db" | head -1)
python3 scripts/prof_db.py $DB stats 15 40 > gpurun_out/r3_norm_gpt2_kernel_stats.txt
rm -rf gpurun_out/p_gpt2
grep -E "total|norm_" gpurun_out/r3_norm_gpt2_kernel_stats.txt | cut -c1-150
for cfg in gemma3-270m-lora gpt2-lora gemma3-270m-lora gpt2-lora; do
  timeout -k 10 300 python3 bench.py --config $cfg >> gpurun_out/norm_bench.jsonl 2> gpurun_out/norm_bench.err || { tail -5 gpurun_out/norm_bench.err; exit 1; }
  tail -1 gpurun_out/norm_bench.jsonl | cut -c1-140
done
