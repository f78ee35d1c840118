#!/bin/bash
# ZeRO-3 after the prescaled-sum reduce-scatter straight into the gradient partition: correctness
# (loopback / RCCL / resume), GPT-2 XL ZeRO-3 (+offload) bench, and batch-64 kernel stats
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 600 python3 -u -m pytest tests/test_engine_dist_gpu.py -x -v --timeout 240 --timeout-method thread \
  -k "zero_stage or zero3 or resume or extra6 or extra7 or extra8" > gpurun_out/r3_z3b_tests.log 2>&1 || { tail -60 gpurun_out/r3_z3b_tests.log; exit 1; }
tail -2 gpurun_out/r3_z3b_tests.log
rm -f gpurun_out/r3_z3b.jsonl
for args in "--config gpt2-xl-zero3" "--config gpt2-xl-zero3-offload" "--config gpt2-xl-zero"; do
  timeout -k 10 300 python3 bench.py $args --steps 10 --warmup 3 >> gpurun_out/r3_z3b.jsonl 2> gpurun_out/r3_z3b.err || { tail -20 gpurun_out/r3_z3b.err; exit 1; }
  tail -1 gpurun_out/r3_z3b.jsonl | cut -c1-300
done
rm -rf gpurun_out/p_z3b
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p_z3b -o run -- mobilefinetuner_amd/bin/gpt2_full_finetune \
  --random_init --synthetic_data --model gpt2-xl --batch_size 64 --seq_len 128 --steps 4 --log_interval 4 --zero_stage 3 \
  > gpurun_out/r3_z3b_prof.log 2>&1 || { tail gpurun_out/r3_z3b_prof.log; exit 1; }
DB=$(find gpurun_out/p_z3b -name "*.db" | head -1)
python3 scripts/prof_db.py $DB stats 4 40 > gpurun_out/r3_z3b_stats.txt
python3 scripts/prof_db.py $DB step adamw_kernel -2 > gpurun_out/r3_z3b_step_trace.txt
rm -rf gpurun_out/p_z3b
