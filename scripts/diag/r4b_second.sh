#!/bin/bash
# round 4 session 2: tests touching the changed kernels (LoRA dy / xty early loads, CE label prefetch,
# norm-fused LoRA u off by default), then the A/B batch and graph-mode kernel stats of both steps
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_lm_head_ce_gpu.py \
  tests/test_lora_dy_gpu.py tests/test_lora_wgrad_gpu.py tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_engine_gemma_gpu.py \
  > gpurun_out/r4b2_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r4b2_tests.log
[ $rc -eq 0 ] || exit 1
bash scripts/diag/r4b_ab.sh || exit 1
A="--random_init --synthetic_data --synthetic_tokens 2000000 --seq_len 128 --batch_size 1024 --steps 14 --log_interval 0 --bench_steps 6 --bench_warmup 4"
rm -rf gpurun_out/p_g2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p_g2 -o run -- mobilefinetuner_amd/bin/gpt2_lora_finetune $A > gpurun_out/r4b2_g2_prof.log 2>&1 || { tail -20 gpurun_out/r4b2_g2_prof.log; exit 1; }
DB=$(find gpurun_out/p_g2 -name "*.db" | head -1)
python3 scripts/prof_db.py $DB stats 10 40 > gpurun_out/r4b2_gpt2_lora_kernel_stats.txt && head -16 gpurun_out/r4b2_gpt2_lora_kernel_stats.txt | cut -c1-150
rm -rf gpurun_out/p_g2
bash scripts/diag/r4_gprof.sh > /dev/null 2>&1
head -24 gpurun_out/r4_gemma_graph_kernel_stats.txt | cut -c1-150
