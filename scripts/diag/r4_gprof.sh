#!/bin/bash
# Gemma-3 step graph under rocprofv3 --kernel-trace (round 3 saw a segfault inside hipGraphLaunch): the
# native fatal-signal handler prints the faulting thread's backtrace; on success the graph-mode kernel
# table is written
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
ARGS="--model gemma3-270m --random_init --synthetic_data --synthetic_tokens 2000000 --batch 256 --seq_len 256 --lora_dropout 0 --targets full"
rm -rf gpurun_out/p_gemma_g
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p_gemma_g -o run -- mobilefinetuner_amd/bin/train_lora_gemma $ARGS --max_steps 12 --log_interval 0 --bench_steps 6 --bench_warmup 4 > gpurun_out/r4_gemma_graph_prof.log 2>&1; rc=$?
echo "gemma graph-mode profile rc=$rc"
grep -A40 "fatal signal" gpurun_out/r4_gemma_graph_prof.log | head -60
grep MFT_BENCH gpurun_out/r4_gemma_graph_prof.log | cut -c1-200
if [ $rc -eq 0 ]; then
  DB=$(find gpurun_out/p_gemma_g -name "*.db" | head -1)
  python3 scripts/prof_db.py $DB stats 10 40 > gpurun_out/r4_gemma_graph_kernel_stats.txt && head -30 gpurun_out/r4_gemma_graph_kernel_stats.txt | cut -c1-160
fi
rm -rf gpurun_out/p_gemma_g
exit 0
