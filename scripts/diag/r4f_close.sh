#!/bin/bash
# round 4 closing validation: the driver's GPU test tier + smoke, every bench config, the headline's and
# Gemma's graph-mode kernel stats
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4f_gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r4f_gpu_tests.log
[ $rc -eq 0 ] || { grep -B3 -A30 "Error\|FAIL" gpurun_out/r4f_gpu_tests.log | head -60; exit 1; }
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4f_smoke.log 2>&1 || { tail -20 gpurun_out/r4f_smoke.log; exit 1; }
tail -2 gpurun_out/r4f_smoke.log | cut -c1-200
: > gpurun_out/r4f_bench.jsonl
for c in gpt2-lora gemma3-270m-lora gpt2-full gpt2-xl-zero gpt2-xl-zero3 gpt2-xl-zero3-offload; do
  timeout -k 10 500 python3 bench.py --config $c --steps 20 --warmup 5 > gpurun_out/r4f_bench_$c.txt 2>&1 || { tail -5 gpurun_out/r4f_bench_$c.txt; exit 1; }
  tail -1 gpurun_out/r4f_bench_$c.txt >> gpurun_out/r4f_bench.jsonl
  tail -1 gpurun_out/r4f_bench_$c.txt | cut -c1-160
done
timeout -k 10 500 python3 bench.py --config gpt2-lora --batch 4 --steps 50 --warmup 10 > gpurun_out/r4f_bench_b4.txt 2>&1 && tail -1 gpurun_out/r4f_bench_b4.txt >> gpurun_out/r4f_bench.jsonl
A="--random_init --synthetic_data --synthetic_tokens 2000000 --seq_len 128 --batch_size 1024 --steps 14 --log_interval 0 --bench_steps 6 --bench_warmup 4"
rm -rf gpurun_out/p_g2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p_g2 -o run -- mobilefinetuner_amd/bin/gpt2_lora_finetune $A > gpurun_out/r4f_g2_prof.log 2>&1 || { tail -5 gpurun_out/r4f_g2_prof.log; exit 1; }
DB=$(find gpurun_out/p_g2 -name "*.db" | head -1)
python3 scripts/prof_db.py $DB stats 10 40 > gpurun_out/r4f_gpt2_lora_kernel_stats.txt && head -12 gpurun_out/r4f_gpt2_lora_kernel_stats.txt | cut -c1-150
rm -rf gpurun_out/p_g2
bash scripts/diag/r4_gprof.sh > /dev/null 2>&1; cp gpurun_out/r4_gemma_graph_kernel_stats.txt gpurun_out/r4f_gemma_graph_kernel_stats.txt 2>/dev/null
head -12 gpurun_out/r4f_gemma_graph_kernel_stats.txt | cut -c1-150
exit 0
