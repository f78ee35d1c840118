#!/bin/bash
# LoRA dy / xty grids sized to one round (no 513th-block tail): LoRA numerics, graph-mode kernel stats of the
# headline, both LoRA benches
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_lora_dy_gpu.py tests/test_lora_wgrad_gpu.py \
  tests/test_kernels_gpu.py -k "lora or rowdot" tests/test_engine_gpu.py > gpurun_out/r4b9_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r4b9_tests.log
[ $rc -eq 0 ] || { grep -B3 -A25 "Error\|FAIL" gpurun_out/r4b9_tests.log | head -50; exit 1; }
A="--random_init --synthetic_data --synthetic_tokens 2000000 --seq_len 128 --batch_size 1024 --steps 14 --log_interval 0 --bench_steps 6 --bench_warmup 4"
rm -rf gpurun_out/p_g2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p_g2 -o run -- mobilefinetuner_amd/bin/gpt2_lora_finetune $A > gpurun_out/r4b9_g2_prof.log 2>&1 || { tail -5 gpurun_out/r4b9_g2_prof.log; exit 1; }
DB=$(find gpurun_out/p_g2 -name "*.db" | head -1)
python3 scripts/prof_db.py $DB stats 10 40 > gpurun_out/r4b9_gpt2_lora_kernel_stats.txt && grep -i "lora\|total" gpurun_out/r4b9_gpt2_lora_kernel_stats.txt | cut -c1-150
rm -rf gpurun_out/p_g2
for r in 1 2; do
  for c in gpt2-lora gemma3-270m-lora; do
    timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 5 2>/dev/null | tail -1 | cut -c1-150
  done
done | tee gpurun_out/r4b9_bench.txt
