#!/bin/bash
# gemm8 LoRA-epilogue data-grads with the B0 fragments kept across phases (KEEPB; the epilogue walks the
# ranks 4 at a time to fit): numerics, then both LoRA steps' graph-mode kernel stats and benches
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 900 python -u -m pytest --maxfail 6 -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_gemm_gpu.py \
  tests/test_engine_gpu.py tests/test_engine_gemma_gpu.py tests/test_parity_full_gpu.py > gpurun_out/r4b11_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r4b11_tests.log
[ $rc -eq 0 ] || grep -A3 "^FAILED\|AssertionError" gpurun_out/r4b11_tests.log | head -40
A="--random_init --synthetic_data --synthetic_tokens 2000000 --seq_len 128 --batch_size 1024 --steps 14 --log_interval 0 --bench_steps 6 --bench_warmup 4"
rm -rf gpurun_out/p_g2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p_g2 -o run -- mobilefinetuner_amd/bin/gpt2_lora_finetune $A > gpurun_out/r4b11_g2_prof.log 2>&1 || { tail -5 gpurun_out/r4b11_g2_prof.log; exit 1; }
DB=$(find gpurun_out/p_g2 -name "*.db" | head -1)
python3 scripts/prof_db.py $DB stats 10 40 > gpurun_out/r4b11_gpt2_lora_kernel_stats.txt && head -3 gpurun_out/r4b11_gpt2_lora_kernel_stats.txt && grep "gemm8_kernel<5" gpurun_out/r4b11_gpt2_lora_kernel_stats.txt | cut -c1-150
rm -rf gpurun_out/p_g2
bash scripts/diag/r4_gprof.sh > /dev/null 2>&1; cp gpurun_out/r4_gemma_graph_kernel_stats.txt gpurun_out/r4b11_gemma_graph_kernel_stats.txt
head -3 gpurun_out/r4b11_gemma_graph_kernel_stats.txt; grep "gemm8_kernel<5" gpurun_out/r4b11_gemma_graph_kernel_stats.txt | cut -c1-150
for r in 1 2; do
  for c in gpt2-lora gemma3-270m-lora; do
    timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 5 2>/dev/null | tail -1 | cut -c1-150
  done
done | tee gpurun_out/r4b11_bench.txt
