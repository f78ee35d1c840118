#!/bin/bash
# kernel stats of the GPT-2 LoRA and Gemma-3 LoRA bench steps (fused LM-head CE) + Gemma bench line
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
prof() {  # tag, steps, bench args...
  local tag=$1 n=$2; shift 2
  rm -rf gpurun_out/p_$tag
  timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/p_$tag -o run -- python3 bench.py --steps $n --warmup 3 "$@" > gpurun_out/p_$tag.log 2>&1 || { tail gpurun_out/p_$tag.log; return 1; }
  DB=$(find gpurun_out/p_$tag -name "*.db" | head -1)
  python3 scripts/prof_db.py $DB stats $((n + 3)) 30 > gpurun_out/${tag}_stats.txt && head -16 gpurun_out/${tag}_stats.txt
  rm -rf gpurun_out/p_$tag
}
prof gpt2 10 && prof gemma 6 --config gemma3-270m-lora && \
timeout -k 10 400 python3 bench.py --config gemma3-270m-lora --steps 20 --warmup 5 > gpurun_out/gemma_bench.jsonl 2>gpurun_out/gemma_bench.err && cat gpurun_out/gemma_bench.jsonl
MFT_CE_BUDGET_GB=40 timeout -k 10 400 python3 bench.py --config gemma3-270m-lora --steps 20 --warmup 5 > gpurun_out/gemma_bench40.jsonl 2>gpurun_out/gemma_bench40.err && cat gpurun_out/gemma_bench40.jsonl
timeout -k 10 300 python3 -m pytest tests/test_lm_head_ce_gpu.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -2
