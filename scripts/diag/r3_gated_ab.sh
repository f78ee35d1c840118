#!/bin/bash
# gated GeGLU kernels with the row-pair mapping: kernel tests, Gemma-3 eager kernel profile, Gemma-3 bench x2
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gated or gelu" > gpurun_out/gated_tests.log 2>&1 || { tail -20 gpurun_out/gated_tests.log; exit 1; }
tail -1 gpurun_out/gated_tests.log
ARGS="--model gemma3-270m --random_init --synthetic_data --synthetic_tokens 2000000 --batch 256 --seq_len 256 --lora_dropout 0 --targets full"
rm -rf gpurun_out/p_gemma
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p_gemma -o run -- mobilefinetuner_amd/bin/train_lora_gemma $ARGS --max_steps 15 --log_interval 0 --bench_steps 10 --bench_warmup 5 --no_graph > gpurun_out/gated_prof.log 2>&1 || { grep -v "^\s*@" gpurun_out/gated_prof.log | tail -5; exit 1; }
DB=$(find gpurun_out/p_gemma -name "*.db" | head -1)
python3 scripts/prof_db.py $DB stats 15 40 > gpurun_out/r3_gated_gemma_kernel_stats.txt
rm -rf gpurun_out/p_gemma
grep -E "total|gated|norm_bwd" gpurun_out/r3_gated_gemma_kernel_stats.txt | cut -c1-150
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --config gemma3-270m-lora >> gpurun_out/gated_bench.jsonl 2> gpurun_out/gated_bench.err || { tail -5 gpurun_out/gated_bench.err; exit 1; }
  tail -1 gpurun_out/gated_bench.jsonl | cut -c1-160
done
