#!/bin/bash
# native ZeRO-3 correctness (loopback 2 ranks == 1 process, RCCL 1-rank in the hipGraph, per-rank
# resume), then native GPT-2 XL ZeRO-2 / ZeRO-3 (+ host-offloaded moments) vs the torch path, and a
# kernel trace of a native ZeRO-3 GPT-2 full step (gathers / reduce-scatters between the kernels)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 900 python3 -u -m pytest tests/test_engine_dist_gpu.py -x -v --timeout 240 --timeout-method thread \
  -k "two_ranks_match or zero3 or resume" > gpurun_out/r3_z3_tests.log 2>&1 || { tail -60 gpurun_out/r3_z3_tests.log; exit 1; }
tail -3 gpurun_out/r3_z3_tests.log
for args in "--config gpt2-xl-zero3" "--config gpt2-xl-zero3-offload" "--config gpt2-xl-zero" \
            "--config gpt2-xl-zero --offload_optimizer" "--config gpt2-xl-zero3 --engine torch"; do
  timeout -k 10 300 python3 bench.py $args --steps 10 --warmup 3 >> gpurun_out/r3_xl_zero.jsonl 2> gpurun_out/r3_xl_zero.err || { tail -20 gpurun_out/r3_xl_zero.err; exit 1; }
  tail -1 gpurun_out/r3_xl_zero.jsonl | cut -c1-400
done
rm -rf gpurun_out/p_z3
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/p_z3 -o run -- mobilefinetuner_amd/bin/gpt2_full_finetune \
  --random_init --synthetic_data --model gpt2-xl --batch_size 32 --seq_len 128 --steps 4 --log_interval 4 --zero_stage 3 \
  > gpurun_out/r3_z3_prof.log 2>&1 || { tail gpurun_out/r3_z3_prof.log; exit 1; }
DB=$(find gpurun_out/p_z3 -name "*.db" | head -1)
python3 scripts/prof_db.py $DB step adamw_kernel -2 > gpurun_out/r3_z3_step_trace.txt
python3 scripts/prof_db.py $DB stats 4 30 > gpurun_out/r3_z3_stats.txt
rm -rf gpurun_out/p_z3
