#!/bin/bash
# every GEMM hand-written (MFT_NT=gemm8 MFT_NN=gemm8: no hipBLASLt kernel in the step) vs the timed per-shape choice
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
rm -f gpurun_out/r3_allg8_ab.txt
for cfg in gpt2-lora gemma3-270m-lora gpt2-full; do
  for v in "MFT_NT=timed" "MFT_NT=gemm8 MFT_NN=gemm8" "MFT_NT=timed" "MFT_NT=gemm8 MFT_NN=gemm8"; do
    env $v timeout -k 10 300 python3 bench.py --config $cfg --steps 20 --warmup 5 > gpurun_out/r3_ag.json 2> gpurun_out/r3_ag.err || { tail -20 gpurun_out/r3_ag.err; exit 1; }
    echo "$cfg [$v]: $(python3 -c 'import json; r=json.load(open("gpurun_out/r3_ag.json")); print(r["value"], r["ms_per_step"])')" | tee -a gpurun_out/r3_allg8_ab.txt
  done
done
