#!/bin/bash
# residual adds in the producing GEMMs' epilogues (GPT-2), the residual gradient through the norm kernels'
# dresid input (resid_out): engine / parity / dist numerics, the headline's kernel stats, benches
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 900 python -u -m pytest --maxfail 6 -q --timeout 300 --timeout-method thread tests/test_engine_gpu.py \
  tests/test_parity_full_gpu.py tests/test_engine_dist_gpu.py tests/test_deterministic_gpu.py > gpurun_out/r4b12_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r4b12_tests.log
[ $rc -eq 0 ] || grep -A3 "^FAILED\|AssertionError" gpurun_out/r4b12_tests.log | head -40
A="--random_init --synthetic_data --synthetic_tokens 2000000 --seq_len 128 --batch_size 1024 --steps 14 --log_interval 0 --bench_steps 6 --bench_warmup 4"
rm -rf gpurun_out/p_g2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p_g2 -o run -- mobilefinetuner_amd/bin/gpt2_lora_finetune $A > gpurun_out/r4b12_g2_prof.log 2>&1 || { tail -5 gpurun_out/r4b12_g2_prof.log; exit 1; }
DB=$(find gpurun_out/p_g2 -name "*.db" | head -1)
python3 scripts/prof_db.py $DB stats 10 40 > gpurun_out/r4b12_gpt2_lora_kernel_stats.txt && head -22 gpurun_out/r4b12_gpt2_lora_kernel_stats.txt | cut -c1-150
rm -rf gpurun_out/p_g2
for r in 1 2; do
  for c in gpt2-lora gpt2-full; do
    timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 5 2>/dev/null | tail -1 | cut -c1-150
  done
done | tee gpurun_out/r4b12_bench.txt
