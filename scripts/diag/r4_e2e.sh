#!/bin/bash
# end-to-end A/B of the gemm8 LDS-staged epilogues (MFT_GEMM8_STREAM=5) and the first-round stagger
# (MFT_G8_STAGGER) on the GPT-2 LoRA headline and Gemma-3, interleaved, 2 rounds
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
out=gpurun_out/r4_e2e.txt; : > $out
for r in 1 2; do
  for cfg in gpt2-lora gemma3-270m-lora; do
    for env in "MFT_GEMM8_STREAM=0" "MFT_GEMM8_STREAM=5" "MFT_GEMM8_STREAM=5 MFT_G8_STAGGER=1200" "MFT_GEMM8_ALL=1 MFT_GEMM8_STREAM=5"; do
      line=$(env $env timeout -k 10 300 python3 bench.py --config $cfg --steps 20 --warmup 5 2>/dev/null | tail -1) || { echo "FAIL $cfg $env" >> $out; exit 1; }
      v=$(echo "$line" | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['value'], r['ms_per_step'])")
      echo "$cfg [$env]: $v" | tee -a $out
    done
  done
done
