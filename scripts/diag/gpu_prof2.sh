#!/bin/bash
# kernel tests touching LoRA, then kernel stats of the GPT-2 LoRA and Gemma-3 LoRA bench steps
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python3 -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_lora_wgrad_gpu.py tests/test_lora_dy_gpu.py > gpurun_out/prof2_tests.log 2>&1 || { tail -20 gpurun_out/prof2_tests.log; exit 1; }
tail -1 gpurun_out/prof2_tests.log
prof() {  # tag, steps, bench args...
  local tag=$1 n=$2; shift 2
  rm -rf gpurun_out/p_$tag
  timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/p_$tag -o run -- python3 bench.py --steps $n --warmup 3 "$@" > gpurun_out/p_$tag.log 2>&1 || { tail gpurun_out/p_$tag.log; return 1; }
  DB=$(find gpurun_out/p_$tag -name "*.db" | head -1)
  python3 scripts/prof_db.py $DB stats $((n + 3)) 40 > gpurun_out/${tag}_stats.txt && head -24 gpurun_out/${tag}_stats.txt | cut -c1-150
  rm -rf gpurun_out/p_$tag
}
prof gpt2 10 && prof gemma 6 --config gemma3-270m-lora
