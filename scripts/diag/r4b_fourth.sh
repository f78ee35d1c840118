#!/bin/bash
# CE anatomy incl. the LDS-staged E epilogue on the CE kernels alone; the reference recipe (4 x 128,
# graph mode) kernel breakdown
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python3 scripts/bench_ce.py > gpurun_out/r4b4_bench_ce.txt 2>&1 || { tail -20 gpurun_out/r4b4_bench_ce.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r4b4_bench_ce.txt
A="--random_init --synthetic_data --synthetic_tokens 200000 --seq_len 128 --batch_size 4 --steps 60 --log_interval 0 --bench_steps 40 --bench_warmup 10"
rm -rf gpurun_out/p_b4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p_b4 -o run -- mobilefinetuner_amd/bin/gpt2_lora_finetune $A > gpurun_out/r4b4_b4_prof.log 2>&1 || { tail -20 gpurun_out/r4b4_b4_prof.log; exit 1; }
grep MFT_BENCH gpurun_out/r4b4_b4_prof.log | cut -c1-200
DB=$(find gpurun_out/p_b4 -name "*.db" | head -1)
python3 scripts/prof_db.py $DB stats 60 40 > gpurun_out/r4b4_b4_kernel_stats.txt && head -30 gpurun_out/r4b4_b4_kernel_stats.txt | cut -c1-150
python3 scripts/prof_db.py $DB step > gpurun_out/r4b4_b4_step.txt 2>&1; tail -2 gpurun_out/r4b4_b4_step.txt | cut -c1-200
rm -rf gpurun_out/p_b4
