#!/bin/bash
# dK/dV offset pair images (half-wave DMA pairs), non-temporal E stores, one-round LoRA dy/xty grids:
# numerics of everything they touch, then attention time + PMC, CE anatomy, the headline's kernel stats, benches
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_engine_gemma_gpu.py tests/test_parity_full_gpu.py tests/test_lm_head_ce_gpu.py tests/test_lora_dy_gpu.py \
  tests/test_lora_wgrad_gpu.py tests/test_engine_gpu.py > gpurun_out/r4b10_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r4b10_tests.log
[ $rc -eq 0 ] || { grep -B3 -A25 "Error\|FAIL" gpurun_out/r4b10_tests.log | head -50; exit 1; }
for r in 1 2; do timeout -k 10 120 python3 scripts/bench_attn256.py 2>&1 | grep -v amdgpu.ids || exit 1; done | tee gpurun_out/r4b10_attn.txt
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc/q -o run -- python3 scripts/diag/attn256_pmc_probe.py > gpurun_out/pmc/q.log 2>&1 || exit 1
DB=$(find gpurun_out/pmc/q -name "*.db" | head -1); python3 scripts/pmc_db.py $DB attn_ | tee gpurun_out/r4b10_attn_pmc.txt; rm -rf gpurun_out/pmc/q
timeout -k 10 300 python3 scripts/bench_ce.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r4b10_bench_ce.txt
A="--random_init --synthetic_data --synthetic_tokens 2000000 --seq_len 128 --batch_size 1024 --steps 14 --log_interval 0 --bench_steps 6 --bench_warmup 4"
rm -rf gpurun_out/p_g2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p_g2 -o run -- mobilefinetuner_amd/bin/gpt2_lora_finetune $A > gpurun_out/r4b10_g2_prof.log 2>&1 || { tail -5 gpurun_out/r4b10_g2_prof.log; exit 1; }
DB=$(find gpurun_out/p_g2 -name "*.db" | head -1)
python3 scripts/prof_db.py $DB stats 10 40 > gpurun_out/r4b10_gpt2_lora_kernel_stats.txt && head -3 gpurun_out/r4b10_gpt2_lora_kernel_stats.txt && grep -i "lora\|gemm8_kernel<7" gpurun_out/r4b10_gpt2_lora_kernel_stats.txt | cut -c1-150
rm -rf gpurun_out/p_g2
for r in 1 2; do
  for c in gpt2-lora gemma3-270m-lora; do
    timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 5 2>/dev/null | tail -1 | cut -c1-150
  done
done | tee gpurun_out/r4b10_bench.txt
